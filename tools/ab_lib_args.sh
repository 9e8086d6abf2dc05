#!/bin/bash
# A/B of (library variant, bench.py arguments) pairs: tools/ab_lib_args.sh OUTDIR "lib:name=ARGS;lib2:name2=ARGS2" [reps]
out=$1; specs=$2; reps=${3:-2}
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
IFS=';' read -ra SP <<< "$specs"
for rep in $(seq 1 $reps); do
  for spec in "${SP[@]}"; do
    lib=${spec%%:*}; rest=${spec#*:}; name=${rest%%=*}; a=${rest#*=}
    cp "variants/lib_$lib.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
    timeout -k 10 300 python bench.py --cpu-sample 0 --no-host-api $a > "$out/b_${lib}_${name}_$rep.json" 2> "$out/b_${lib}_${name}_$rep.err" || { echo "$lib $name failed"; tail -3 "$out/b_${lib}_${name}_$rep.err"; cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so; exit 1; }
    echo "$lib $name $(python -c "import json; d=json.load(open('$out/b_${lib}_${name}_$rep.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items() if v})")"
  done
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
