#!/bin/bash
# round 4: C5 tests on the default build, C5 traces of two variants, C5 PMC
set -o pipefail
out=gpurun_out/r04l
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c5.py -m gpu > "$out/c5_tests.log" 2>&1 \
  || { echo "c5 tests failed"; grep -E "FAIL|Error|assert" "$out/c5_tests.log" | head -20; exit 1; }
tail -1 "$out/c5_tests.log"
bash tools/c5_trace_variants.sh "$out/c5" "cur ipb1 ipb4" || exit 1
