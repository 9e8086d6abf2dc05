#!/bin/bash
# A/B of prebuilt library variants (variants/lib_*.so) x sub-batch stream counts.
# usage: tools/ab_variants.sh OUTDIR "v1 v2 ..." "s1 s2 ..."
set -e
out=$1; vars=$2; streams=${3:-"1 2"}
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  for s in $streams; do
    timeout -k 10 300 python bench.py --cpu-sample 0 --streams "$s" --steps 20 > "$out/b_${v}_s$s.json" 2> "$out/b_${v}_s$s.err"
    echo "$v s=$s $(python -c "import json,sys; d=json.load(open('$out/b_${v}_s$s.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items() if v})")"
  done
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
