#!/bin/bash
# The matcher-latency harness under rocprofv3 --kernel-trace --stats (tools
# only): the per-kernel durations behind each host call's latency, the upload
# and the dframe forms (tests/native/matcher_latency).
# usage: tools/gpu_lat_trace.sh <tag> [reps] [library]   outputs under gpurun_out/<tag>/ (lat_*<library stem>)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
reps=${2:-50}
lib=${3:-orb_slam3_vio_fixes_amd/liborb_mi355x.so}
sfx=""; [ -n "$3" ] && sfx=_$(basename $3 .so)
d=$(mktemp -d)
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
import bench
from orb_slam3_vio_fixes_amd import synth
print(bench.matcher_inputs(synth.global_sequence(752, 480, 0, 2, config=2), '$d'))
" > $out/lat_inputs.log 2>&1 || { echo inputs failed; tail $out/lat_inputs.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lat_trace$sfx -o run -- \
    ./tests/native/bin/matcher_latency $lib orbm $d $reps \
    > $out/lat_trace$sfx.json 2> $out/lat_trace$sfx.err || { echo trace failed; tail $out/lat_trace$sfx.err; exit 1; }
python tools/kstats.py $out/lat_trace$sfx/run_kernel_trace.csv > $out/lat_kstats$sfx.txt
head -30 $out/lat_kstats$sfx.txt
