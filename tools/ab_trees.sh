#!/bin/bash
# Same-box A/B of two whole trees (e.g. a git worktree of an earlier round
# under variants/) on one bench workload.
# usage: tools/ab_trees.sh OUTDIR OTHER_TREE "bench args" [reps]
set -e
out=$(realpath -m "$1"); other=$2; args=$3; reps=${4:-2}
mkdir -p "$out"
root=$(pwd)
for i in $(seq 1 "$reps"); do
  for t in cur other; do
    d=$root; [ $t = other ] && d=$other
    (cd "$d" && timeout -k 10 300 python bench.py $args > "$out/${t}_$i.json" 2> "$out/${t}_$i.err")
    echo "$t $i $(python -c "import json; d=json.loads(open('$out/${t}_$i.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['stage_ms'].items() if x})")"
  done
done
