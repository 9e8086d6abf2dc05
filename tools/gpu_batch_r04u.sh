#!/bin/bash
# r04u: k_quadtree keys in registers (ORB_QT_KREG keys per thread) A/B.
set -o pipefail
out=gpurun_out/r04u
mkdir -p "$out"
for v in q8 q6; do
  bash tools/variant_tests.sh "$out" $v tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_sort.py tests/test_gpu_streams.py -m gpu || exit 1
done
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "q0 q8 q6 q4 q0 q8 q6 q4" || exit 1
bash tools/ab_variants.sh "$out/ab" "q0 q8 q6 q0 q8 q6" "1" || exit 1
