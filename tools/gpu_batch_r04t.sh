#!/bin/bash
# r04t: k_quadtree phase profile (-DORB_QT_TIMING build swapped in).
set -o pipefail
out=gpurun_out/r04t
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
cp variants/lib_qtt.so orb_slam3_vio_fixes_amd/liborb_mi355x.so
timeout -k 10 300 python tools/fast_phases.py > "$out/qt_phases.txt" 2>&1; rc=$?
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
cat "$out/qt_phases.txt"
exit $rc
