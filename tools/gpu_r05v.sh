#!/bin/bash
# FAST cells per wave 3 / 4 vs 2 with the row loads
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05v "lib=variants/lib_cpw3.so" "tests=extractor" "lib=variants/lib_cpw4.so" "tests=extractor" \
  "lib=variants/lib_base.so" "bench=$B" "lib=variants/lib_cpw3.so" "bench=$B" "lib=variants/lib_cpw4.so" "bench=$B" \
  "lib=variants/lib_base.so" "bench=$B" "lib=variants/lib_cpw3.so" "bench=$B" "lib=variants/lib_cpw4.so" "bench=$B"
