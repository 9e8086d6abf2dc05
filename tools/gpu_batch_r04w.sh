#!/bin/bash
# r04w: k_describe rBRIEF test loop unrolled by 2 (and with 8 slots a wave) A/B.
set -o pipefail
out=gpurun_out/r04w
mkdir -p "$out"
bash tools/variant_tests.sh "$out" q2 tests/test_gpu_extractor.py -m gpu || exit 1
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "cur q2 q2s8 cur q2 q2s8" || exit 1
bash tools/ab_variants.sh "$out/ab" "cur q2 q2s8 cur q2 q2s8" "1" || exit 1
