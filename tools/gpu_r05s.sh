#!/bin/bash
# k_describe with row loads: pattern floats in registers (PATF) and two patches in flight (PF2) vs default
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05s "lib=variants/lib_descpatf.so" "tests=extractor" "lib=variants/lib_descpf2.so" "tests=extractor" \
  "lib=variants/lib_descrow.so" "bench=$B" "lib=variants/lib_descpatf.so" "bench=$B" "lib=variants/lib_descpf2.so" "bench=$B" \
  "lib=variants/lib_descrow.so" "bench=$B" "lib=variants/lib_descpatf.so" "bench=$B" "lib=variants/lib_descpf2.so" "bench=$B"
