#!/bin/bash
# Phase profiles (tools/fast_phases.py) of timing-instrumented library variants.
# usage: tools/phase_ab.sh OUTDIR "v1 v2 ..."   (variants/lib_<v>.so built with -DORB_*_TIMING)
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  echo "== $v"
  timeout -k 10 120 python tools/fast_phases.py > "$out/$v.txt" 2>&1 || { echo "$v failed"; tail -5 "$out/$v.txt"; cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so; exit 1; }
  cat "$out/$v.txt"
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
