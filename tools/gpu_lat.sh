#!/bin/bash
# matcher-latency harness on the GPU (tools only): inputs from bench.matcher_inputs, one JSON line
# usage: tools/gpu_lat.sh <tag> [reps]
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
d=$(mktemp -d)
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
import bench
from orb_slam3_vio_fixes_amd import synth
print(bench.matcher_inputs(synth.global_sequence(752, 480, 0, 2, config=2), '$d'))
" > $out/lat_inputs.log 2>&1 || { echo inputs failed; tail $out/lat_inputs.log; exit 1; }
timeout -k 10 200 ./tests/native/bin/matcher_latency orb_slam3_vio_fixes_amd/liborb_mi355x.so orbm $d ${2:-200} > $out/lat.json 2> $out/lat.err || { echo lat failed; tail $out/lat.err; exit 1; }
cat $out/lat.json
