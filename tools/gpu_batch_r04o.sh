#!/bin/bash
# r04o: k_describe border patches with batched reflected byte loads (A/B).
set -o pipefail
out=gpurun_out/r04o
mkdir -p "$out"
for v in db6 db10; do
  bash tools/variant_tests.sh "$out" $v tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_adapter.py -m gpu || exit 1
done
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "db0 db6 db10 db0 db6 db10" || exit 1
bash tools/ab_variants.sh "$out/ab" "db0 db6 db10 db0 db6 db10" "1" || exit 1
