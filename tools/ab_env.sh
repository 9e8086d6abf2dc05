#!/bin/bash
# A/B of one library under environment settings: tools/ab_env.sh OUTDIR "NAME=ENV ..." (ENV "-" = none)
# e.g. tools/ab_env.sh gpurun_out/x "lds40=- lds0=ORB_QT_LDS_KB=0"
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for spec in $1; do
    name=${spec%%=*}; envs=${spec#*=}
    [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 300 python bench.py --cpu-sample 0 --steps 20 > "$out/b_${name}_$rep.json" 2> "$out/b_${name}_$rep.err" || { echo "$name failed"; tail -3 "$out/b_${name}_$rep.err"; exit 1; }
    echo "$name $(python -c "import json; d=json.load(open('$out/b_${name}_$rep.json')); print(round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items() if v})")"
  done
done
