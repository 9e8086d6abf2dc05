#!/bin/bash
# r04n: FAST cell-loop landing (mad24) and row decode (v_rcp) A/B.
set -o pipefail
out=gpurun_out/r04n
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_configs.py tests/test_gpu_adapter.py tests/test_gpu_streams.py -m gpu > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "old new old new" || exit 1
bash tools/ab_variants.sh "$out/ab" "old new old new" "1" || exit 1
