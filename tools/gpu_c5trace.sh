#!/bin/bash
# C5 kernel trace (stated map) -> kstats
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --workload c5 --cpu-sample 0 > $out/c5.json 2> $out/c5.err || { echo trace failed; tail -5 $out/c5.err; exit 1; }
python tools/kstats.py $out/trace/run_kernel_trace.csv --csv $out/kstats.csv > $out/kstats.txt
head -20 $out/kstats.txt
