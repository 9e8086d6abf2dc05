#!/bin/bash
# r04q: k_fast_cells launched per level range (small-celled levels at 5 waves a SIMD) A/B.
set -o pipefail
out=gpurun_out/r04q
mkdir -p "$out"
bash tools/variant_tests.sh "$out" split tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_adapter.py tests/test_gpu_streams.py -m gpu || exit 1
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "nosplit split nosplit split" || exit 1
bash tools/ab_variants.sh "$out/ab" "nosplit split nosplit split" "1" || exit 1
