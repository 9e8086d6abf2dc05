#!/bin/bash
# The matcher-latency harness without the profiler (tools only): latencies as
# the host sees them, with whatever diagnostics the environment asks for
# (options: orb_debug_set_option pairs, e.g. 9=30 = ORB_OPT_BOW_TRACE: the
# 30th BoW dframe call prints its per-wave checkpoints).
# usage: tools/gpu_lat_run.sh <tag> [reps] [library] [opt=value,...]   outputs under gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
reps=${2:-50}
lib=${3:-orb_slam3_vio_fixes_amd/liborb_mi355x.so}
opts=$4
sfx=""; [ -n "$3" ] && sfx=_$(basename $3 .so)
d=$(mktemp -d)
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
import bench
from orb_slam3_vio_fixes_amd import synth
print(bench.matcher_inputs(synth.global_sequence(752, 480, 0, 2, config=2), '$d'))
" > $out/lat_inputs.log 2>&1 || { echo inputs failed; tail $out/lat_inputs.log; exit 1; }
timeout -k 10 120 ./tests/native/bin/matcher_latency $lib orbm $d $reps $opts > $out/lat_run$sfx.json 2> $out/lat_run$sfx.err \
    || { echo run failed; tail $out/lat_run$sfx.err; exit 1; }
tail -c 600 $out/lat_run$sfx.json
