#!/bin/bash
# k_sfi_resolve time of prebuilt variants (variants/lib_<v>.so) on the
# SearchForInitialization batch alone (tools/sfi_counts.py under a kernel trace).
# usage: tools/gpu_sfi_ab.sh OUTDIR "v1 v2 ..."
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
export TMPDIR=/tmp
rc=0
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v" -o run -- python3 tools/sfi_counts.py > "$out/$v.log" 2>&1 || { rc=1; echo "$v failed"; break; }
  echo "$v $(grep -h 'k_sfi_resolve\|k_sfi_topk' "$out/$v/run_kernel_stats.csv" | cut -d, -f1,4 | tr '\n' ' ')"
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
exit $rc
