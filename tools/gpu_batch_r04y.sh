#!/bin/bash
# r04y: k_fast_cells compact LDS (realigned ROI rows, shared map border) A/B: fixed pitch 13 (c) and per-cell pitch (cd).
set -o pipefail
out=gpurun_out/r04y
mkdir -p "$out"
for v in c cd; do
  bash tools/variant_tests.sh "$out" $v tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_adapter.py tests/test_gpu_streams.py -m gpu || exit 1
done
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "base c cd base c cd" || exit 1
bash tools/ab_variants.sh "$out/ab" "base c cd base c cd" "1" || exit 1
