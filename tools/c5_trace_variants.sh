#!/bin/bash
# C5 bench (ms/query, parity) and its kernel-trace stats for library variants.
# usage: tools/c5_trace_variants.sh OUTDIR "v1 v2 ..."
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
export TMPDIR=/tmp
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
rc=0
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  mkdir -p "$out/$v"
  timeout -k 10 300 python bench.py --workload c5 --cpu-sample 0 > "$out/$v/c5.json" 2> "$out/$v/c5.err" || { echo "$v bench failed"; tail -5 "$out/$v/c5.err"; rc=1; break; }
  echo "$v $(python -c "import json; d=json.load(open('$out/$v/c5.json')); print(round(d['ms_per_query'],3), d.get('parity'))")"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v/trace" -o run -- python3 bench.py --workload c5 --cpu-sample 0 --steps 3 --warmup 1 > "$out/$v/trace.log" 2>&1 || { echo "$v trace failed"; tail -5 "$out/$v/trace.log"; rc=1; break; }
  python tools/kstats.py "$out/$v/trace/run_kernel_trace.csv" --csv "$out/$v/kernel_stats_by_grid.csv" > "$out/$v/kstats.txt"
  head -12 "$out/$v/kstats.txt"
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
exit $rc
