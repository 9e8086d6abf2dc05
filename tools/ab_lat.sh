#!/bin/bash
# A/B of prebuilt library variants (variants/lib_*.so) on the per-call matcher latencies (tools/gpu_lat.sh).
# usage: tools/ab_lat.sh <tag> "v1 v2 ..." [reps]
set -o pipefail
tag=$1; vars=$2; reps=${3:-300}
LIB=orb_slam3_vio_fixes_amd/liborb_mi355x.so
mkdir -p gpurun_out/$tag
cp $LIB gpurun_out/$tag/.default.so
i=0
for v in $vars; do
  i=$((i+1))
  cp variants/lib_$v.so $LIB
  bash tools/gpu_lat.sh ${tag}/${v}_$i $reps - > gpurun_out/$tag/${v}_$i.txt 2>&1 || { echo "$v failed"; tail -5 gpurun_out/$tag/${v}_$i.txt; break; }
  python3 -c "
import json; d=json.load(open('gpurun_out/$tag/${v}_$i/lat_1.json'))
print('$v', {k: v['median_us'] for k, v in d.items() if 'median_us' in v}, 'mps p2', d['search_by_projection_mps_stats'].get('p2_decide_clk'), d['search_by_projection_mps_stats'].get('phase2_clk'))"
done
cp gpurun_out/$tag/.default.so $LIB
