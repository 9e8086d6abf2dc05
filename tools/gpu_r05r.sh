#!/bin/bash
# k_describe at 5 waves a SIMD (20 VGPR spills) vs 4, both with row loads
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05r "lib=variants/lib_desc5.so" "tests=extractor or configs" \
  "bench=$B" "lib=variants/lib_descrow.so" "bench=$B" "lib=variants/lib_desc5.so" "bench=$B" "lib=variants/lib_descrow.so" "bench=$B"
