#!/bin/bash
# r04zz: k_fast_cells phase profile (-DORB_FAST_TIMING build swapped in).
set -o pipefail
out=gpurun_out/r04zz
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
cp variants/lib_fastt.so orb_slam3_vio_fixes_amd/liborb_mi355x.so
timeout -k 10 300 python tools/fast_phases.py > "$out/fast_phases.txt" 2>&1; rc=$?
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
cat "$out/fast_phases.txt"
exit $rc
