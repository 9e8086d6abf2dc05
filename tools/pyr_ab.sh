#!/bin/bash
# A/B of k_pyramid launch groupings (ORB_PYR_GROUPS) and the legacy per-level
# kernel on one box: the pyramid stage time of the default bench.
# usage: tools/pyr_ab.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/pyr_ab}
mkdir -p "$out"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --cpu-sample 0 --no-host-api --steps 30 > "$out/$tag.json" 2> "$out/$tag.err" || { echo "$tag failed"; tail -5 "$out/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$out/$tag.json')); print('$tag', round(d['value']), round(d['stage_ms']['pyramid']*1e3,1), 'us pyramid')"
}
run default X=1
run legacy ORB_PYR_LEGACY=1
run g_0-3-7 ORB_PYR_GROUPS=0-3:16,3-7:32
run g_0-2-5-7 ORB_PYR_GROUPS=0-2:24,2-5:24,5-7:32
run g_0-4-7_24 ORB_PYR_GROUPS=0-4:24,4-7:32
run g_0-7 ORB_PYR_GROUPS=0-7:16
run g_0-7_24 ORB_PYR_GROUPS=0-7:24
run default2 X=1
