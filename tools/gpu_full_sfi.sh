#!/bin/bash
# Every GPU test, then kernel-trace times of library variants (SFI alone).
set -o pipefail
tag=$1; vars=$2
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests -m gpu > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
bash tools/prof_variants.sh "$out/prof" "$vars"
