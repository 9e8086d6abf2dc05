#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel for library variants (one --pmc pass each).
# usage: tools/pmc_fetch_ab.sh OUTDIR "v1 v2 ..."
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
export TMPDIR=/tmp
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/$v/p_$grp" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-host-api --no-profile > "$out/$v.$grp.log" 2>&1 || { echo "$v $grp failed"; cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so; exit 1; }
  done
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
echo done
