#!/bin/bash
# GPU tests run against a library variant (variants/lib_<v>.so swapped in).
# usage: tools/variant_tests.sh OUTDIR VARIANT PYTEST_ARGS...
set -o pipefail
out=$1; v=$2; shift 2
mkdir -p "$out"
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > "$out/tests_$v.log" 2>&1
rc=$?
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
echo "$v: $(tail -1 "$out/tests_$v.log")"
exit $rc
