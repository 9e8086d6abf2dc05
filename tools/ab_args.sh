#!/bin/bash
# A/B of bench.py argument sets on one library: tools/ab_args.sh OUTDIR "name=ARGS;name2=ARGS2" [reps]
# (ARGS with spaces: separate sets by ';', e.g. "o1=--overlap 1;o2=--overlap 2")
out=$1; specs=$2; reps=${3:-2}
mkdir -p "$out"
IFS=';' read -ra SP <<< "$specs"
for rep in $(seq 1 $reps); do
  for spec in "${SP[@]}"; do
    name=${spec%%=*}; a=${spec#*=}
    timeout -k 10 300 python bench.py --cpu-sample 0 --no-host-api $a > "$out/b_${name}_$rep.json" 2> "$out/b_${name}_$rep.err" || { echo "$name failed"; tail -3 "$out/b_${name}_$rep.err"; exit 1; }
    echo "$name $(python -c "import json; d=json.load(open('$out/b_${name}_$rep.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items() if v})")"
  done
done
