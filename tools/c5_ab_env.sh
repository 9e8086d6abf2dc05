#!/bin/bash
# C5 parity tests, then the C5 bench under each "VAR=value" setting given.
# usage: tools/c5_ab_env.sh OUTDIR "ORBM_X=1 ORBM_X=2 ..."
set -o pipefail
out=$1; mkdir -p "$out"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for kv in $2; do
  env $kv timeout -k 10 300 python bench.py --workload c5 --cpu-sample 0 > "$out/c5_$kv.json" 2> "$out/c5_$kv.err" || { echo "$kv failed"; tail -5 "$out/c5_$kv.err"; exit 1; }
  echo "$kv $(python -c "import json; d=json.load(open('$out/c5_$kv.json')); print(round(d['ms_per_query'],3))")"
done
