#!/bin/bash
# A/B of prebuilt library variants (variants/lib_*.so) on the C5 bench.
# usage: tools/ab_c5.sh OUTDIR "v1 v2 ..."
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  timeout -k 10 300 python bench.py --workload c5 --cpu-sample 0 > "$out/c5_$v.json" 2> "$out/c5_$v.err" || { echo "$v failed"; tail -5 "$out/c5_$v.err"; break; }
  echo "$v $(python -c "import json; d=json.load(open('$out/c5_$v.json')); print(round(d['ms_per_query'],3), d.get('parity'))")"
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
