#!/bin/bash
# A/B of prebuilt library variants on C4 (bench.py --workload c4) and C2.
# usage: tools/ab_c4.sh OUTDIR "v1 v2 ..."
set -e
out=$1; vars=$2
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  timeout -k 10 300 python bench.py --workload c4 > "$out/c4_$v.json" 2> "$out/c4_$v.err"
  timeout -k 10 300 python bench.py --cpu-sample 0 --steps 20 > "$out/c2_$v.json" 2> "$out/c2_$v.err"
  echo "$v c4 $(python -c "import json; d=json.load(open('$out/c4_$v.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['stage_ms'].items()})")"
  echo "$v c2 $(python -c "import json; d=json.load(open('$out/c2_$v.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['stage_ms'].items() if x})")"
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
