#!/bin/bash
# r04s: k_describe at 5 waves a SIMD (96 VGPRs, a few spills) A/B.
set -o pipefail
out=gpurun_out/r04s
mkdir -p "$out"
bash tools/variant_tests.sh "$out" w5b4 tests/test_gpu_extractor.py -m gpu || exit 1
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "cur w5b4 w5b2 cur w5b4 w5b2" || exit 1
bash tools/ab_variants.sh "$out/ab" "cur w5b4 w5b2 cur w5b4 w5b2" "1" || exit 1
