#!/bin/bash
# k_describe: patch rows loaded one row per lane (3 x 16 B) vs the 516-dword spread; tests on the variant + bench A/B
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05q "lib=variants/lib_descrow.so" "tests=extractor or configs or math or adapter or smoke" \
  "bench=$B" "lib=variants/lib_descbase.so" "bench=$B" "lib=variants/lib_descrow.so" "bench=$B" "lib=variants/lib_descbase.so" "bench=$B"
