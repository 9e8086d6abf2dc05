#!/bin/bash
# matcher-latency harness on the GPU (tools only): inputs from bench.matcher_inputs, one JSON line per option set
# usage: tools/gpu_lat.sh <tag> [reps] [option set ...]   (an option set: "opt=value,..." or "-" for the defaults)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
reps=${2:-200}; shift; shift
sets=("$@"); [ ${#sets[@]} -eq 0 ] && sets=(-)
d=$(mktemp -d)
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
import bench
from orb_slam3_vio_fixes_amd import synth
print(bench.matcher_inputs(synth.global_sequence(752, 480, 0, 2, config=2), '$d'))
" > $out/lat_inputs.log 2>&1 || { echo inputs failed; tail $out/lat_inputs.log; exit 1; }
i=0
for o in "${sets[@]}"; do
  i=$((i+1)); extra=(); [ "$o" != "-" ] && extra=("$o")
  timeout -k 10 200 ./tests/native/bin/matcher_latency orb_slam3_vio_fixes_amd/liborb_mi355x.so orbm $d $reps "${extra[@]}" \
    > $out/lat_$i.json 2> $out/lat_$i.err || { echo lat $o failed; tail $out/lat_$i.err; exit 1; }
  echo "[$o] $(cat $out/lat_$i.json)"
done
if [ -x tools/_latency_floor ]; then
  timeout -k 10 60 ./tools/_latency_floor > $out/latency_floor.txt 2>&1 || { echo floor failed; exit 1; }
  cat $out/latency_floor.txt
fi
