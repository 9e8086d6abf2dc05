#!/bin/bash
# GPU validation of the in-tree library on the extractor suites, then a same-box A/B of variants.
# usage: tools/r03_validate.sh <tag> "<variants>"
set -o pipefail
tag=$1; vars=$2
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
bash tools/ab_variants.sh "$out/ab" "$vars $vars" "1"
