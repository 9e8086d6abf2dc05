#!/bin/bash
# round 4: C5 tests, trace and PMC passes on the default build
set -o pipefail
out=gpurun_out/r04q
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c5.py -m gpu > "$out/c5_tests.log" 2>&1 \
  || { echo "c5 tests failed"; grep -E "FAIL|Error|assert" "$out/c5_tests.log" | head -20; exit 1; }
tail -1 "$out/c5_tests.log"
bash tools/c5_trace_variants.sh "$out/c5" "cur" || exit 1
bash tools/pmc_c5.sh "$out/pmc_c5" && python tools/pmc_summary.py "$out/pmc_c5" --csv "$out/pmc_c5/summary.csv" > "$out/pmc_c5/summary.txt"
grep -E "bowk" "$out/pmc_c5/summary.txt" | cut -c1-420
