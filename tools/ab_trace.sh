#!/bin/bash
# Kernel-trace A/B of prebuilt library variants: per variant one rocprofv3
# --kernel-trace run of a short bench, the profiled pass's per-kernel stats.
# usage: tools/ab_trace.sh OUTDIR "v1 v2 ..." [kernel regex]
set -o pipefail
out=$1; vars=$2; pat=${3:-.}
mkdir -p "$out"
export TMPDIR=/tmp
LIB=orb_slam3_vio_fixes_amd/liborb_mi355x.so
cp $LIB "$out/.default.so"
i=0
for v in $vars; do
  i=$((i+1))
  cp "variants/lib_$v.so" $LIB
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/t_${v}_$i" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-host-api > "$out/t_${v}_$i.json" 2> "$out/t_${v}_$i.err" || { echo "$v trace failed"; tail -5 "$out/t_${v}_$i.err"; break; }
  python tools/kstats.py "$out/t_${v}_$i/run_kernel_trace.csv" --last 10 > "$out/k_${v}_$i.txt"
  echo "== $v"; grep -E "$pat" "$out/k_${v}_$i.txt" || true
done
cp "$out/.default.so" $LIB
