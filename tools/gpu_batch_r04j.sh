#!/bin/bash
# round 4: every GPU test on the default build, then the C5 (K=4 / K=2) and
# FAST (lerp / u16 pre-test) variant measurements
set -o pipefail
out=gpurun_out/r04j
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > "$out/gpu_tests.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" "$out/gpu_tests.log" | head -20; exit 1; }
tail -1 "$out/gpu_tests.log"
bash tools/ab_variants.sh "$out/ab" "cur nolerp" "1" || exit 1
bash tools/c5_trace_variants.sh "$out/c5" "cur k2" || exit 1
bash tools/variant_tests.sh "$out" k2 tests/test_gpu_c5.py -m gpu -k "adversarial or resolve_forms or every_keyframe" || exit 1
bash tools/prof_variants.sh "$out/prof" "cur nolerp"
