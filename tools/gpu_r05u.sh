#!/bin/bash
# k_fast_cells row loads: 16-byte groups (ROWLOAD=2) vs dword loads (ROWLOAD=1, default)
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05u "lib=variants/lib_fastrow2.so" "tests=extractor or configs or fast or pretest" \
  "bench=$B" "lib=variants/lib_fastrow1.so" "bench=$B" "lib=variants/lib_fastrow2.so" "bench=$B" "lib=variants/lib_fastrow1.so" "bench=$B"
