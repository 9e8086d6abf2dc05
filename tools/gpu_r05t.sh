#!/bin/bash
# k_fast_cells: ROI rows fetched one row per lane (16-dword form) vs the spread; tests on the variant + bench A/B
set -o pipefail
B="--cpu-sample 0 --no-host-api"
bash tools/gpu_session.sh r05t "lib=variants/lib_fastrow.so" "tests=extractor or configs or fast or pretest or adapter or smoke" \
  "bench=$B" "lib=variants/lib_descrow.so" "bench=$B" "lib=variants/lib_fastrow.so" "bench=$B" "lib=variants/lib_descrow.so" "bench=$B"
