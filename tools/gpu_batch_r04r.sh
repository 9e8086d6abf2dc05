#!/bin/bash
# r04r: k_fast_cells item list in the score map's bytes (18 waves a CU) A/B, and with the level split.
set -o pipefail
out=gpurun_out/r04r
mkdir -p "$out"
for v in alias asplit; do
  bash tools/variant_tests.sh "$out" $v tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_adapter.py tests/test_gpu_streams.py -m gpu || exit 1
done
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "base alias asplit base alias asplit" || exit 1
bash tools/ab_variants.sh "$out/ab" "base alias asplit base alias asplit" "1" || exit 1
