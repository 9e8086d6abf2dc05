#!/bin/bash
# SearchForInitialization parity suites, then kernel-trace times of library variants.
# usage: tools/gpu_sfi_check.sh <tag> "v1 v2 ..."
set -o pipefail
tag=$1; vars=$2
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_matcher.py tests/test_gpu_configs.py tests/test_gpu_sharding.py -m gpu > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
bash tools/prof_variants.sh "$out/prof" "$vars"
