#!/bin/bash
# r05f: C5 tests (incl. the low-overlap map), both C5 bench maps, the matcher-latency harness under a kernel trace
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r05f "tests=c5" "bench=--workload c5" "bench=--workload c5 --near-frac 0.1" || exit 1
out=gpurun_out/r05f
d=$(mktemp -d)
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
import bench, numpy as np
from orb_slam3_vio_fixes_amd import synth
fr = synth.global_sequence(752, 480, 0, 2, config=2)
print(bench.matcher_inputs(fr, '$d'))
" > $out/lat_inputs.log 2>&1 || { echo inputs failed; tail $out/lat_inputs.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lattrace -o run -- ./tests/native/bin/matcher_latency orb_slam3_vio_fixes_amd/liborb_mi355x.so orbm $d 200 > $out/lat.json 2> $out/lat.err || { echo lat failed; tail $out/lat.err; exit 1; }
cat $out/lat.json
python tools/kstats.py $out/lattrace/run_kernel_trace.csv > $out/lat_kstats.txt
head -20 $out/lat_kstats.txt
