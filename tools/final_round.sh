#!/bin/bash
# End-of-milestone GPU session: tests, bench, rocprof stats, PMC passes (round_profile.sh), then the C5 line and its kernel trace.
# usage: tools/final_round.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
bash tools/round_profile.sh $1 || exit 1
out=gpurun_out/$1
timeout -k 10 400 python bench.py --workload c5 > $out/c5_bench.json 2> $out/c5.err || { echo c5 failed; tail -5 $out/c5.err; exit 1; }
python -c "import json; d=json.load(open('$out/c5_bench.json')); print('c5', d['ms_per_query'], d.get('parity'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c5trace -o run -- python3 bench.py --workload c5 --cpu-sample 0 > $out/c5_prof.json 2> $out/c5prof.err || { echo c5 prof failed; exit 1; }
python tools/kstats.py $out/c5trace/run_kernel_trace.csv > $out/c5_kstats.txt
echo alldone
