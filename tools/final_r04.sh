#!/bin/bash
# End-of-round GPU session (round 4): tests, bench, rocprof stats, PMC passes (round_profile.sh),
# then the C5 line with its kernel trace and the C3/C4 lines.
# usage: tools/final_r04.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
bash tools/round_profile.sh $1 || exit 1
out=gpurun_out/$1
timeout -k 10 400 python bench.py --workload c5 > $out/c5_bench.json 2> $out/c5.err || { echo c5 failed; tail -5 $out/c5.err; exit 1; }
python -c "import json; d=json.load(open('$out/c5_bench.json')); print('c5', d.get('ms_per_query'), d.get('parity'))"
timeout -k 10 300 python bench.py --workload c3 > $out/c3_bench.json 2> $out/c3.err || { echo c3 failed; tail -5 $out/c3.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 > $out/c4_bench.json 2> $out/c4.err || { echo c4 failed; tail -5 $out/c4.err; exit 1; }
python -c "
import json
for w in ('c3', 'c4'):
    d = json.load(open('$out/' + w + '_bench.json')); print(w, d.get('value'), d.get('unit'), d.get('parity'))"
# the C5 map variant with invalid MapPoints and varied overlap:
# 4000 of the query's features per keyframe, 90 % valid
timeout -k 10 400 python bench.py --workload c5 --per-kf 4000 --valid-frac 0.9 > $out/c5v_bench.json 2> $out/c5v.err || { echo c5v failed; tail -5 $out/c5v.err; exit 1; }
python -c "import json; d=json.load(open('$out/c5v_bench.json')); print('c5v', d.get('ms_per_query'), d.get('mappoints_valid_frac'), d.get('parity'))"
echo alldone
