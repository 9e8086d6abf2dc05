#!/bin/bash
# Round-5 record session B: C5 on the stated map and on the low-overlap map, C3, C4,
# and the per-call matcher latencies.
# usage: tools/final_r05b.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload c5 > $out/c5_bench.json 2> $out/c5.err || { echo c5 failed; tail -5 $out/c5.err; exit 1; }
python tools/bench_brief.py $out/c5_bench.json
timeout -k 10 400 python bench.py --workload c5 --near-frac 0.1 > $out/c5low_bench.json 2> $out/c5low.err || { echo c5low failed; tail -5 $out/c5low.err; exit 1; }
python tools/bench_brief.py $out/c5low_bench.json
timeout -k 10 300 python bench.py --workload c3 > $out/c3_bench.json 2> $out/c3.err || { echo c3 failed; tail -5 $out/c3.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 > $out/c4_bench.json 2> $out/c4.err || { echo c4 failed; tail -5 $out/c4.err; exit 1; }
python -c "
import json
for w in ('c3', 'c4'):
    d = json.load(open('$out/' + w + '_bench.json')); print(w, d.get('value'), d.get('unit'), d.get('parity'))"
bash tools/gpu_lat.sh $tag 500 - || exit 1
echo alldone
