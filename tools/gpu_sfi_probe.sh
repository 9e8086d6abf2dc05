#!/bin/bash
# SearchForInitialization walk probe: phase cycles and counts from the
# -DORB_SFI_COUNT variant (variants/lib_sfic.so), then the variant's kernel
# trace (its k_sfi_resolve time against the product's shows the stamps' cost).
# usage: tools/gpu_sfi_probe.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/sfi_probe}
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
cp variants/lib_sfic.so orb_slam3_vio_fixes_amd/liborb_mi355x.so
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/sfi_counts.py > "$out/counts.txt" 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 tools/sfi_counts.py > "$out/prof.log" 2>&1
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
cat "$out/counts.txt"
exit $rc
