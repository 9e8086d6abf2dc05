#!/bin/bash
# tools/gpu_check.sh, then a same-box A/B of library variants (variants/lib_<v>.so)
# usage: tools/gpu_check_ab.sh <tag> "v1 v2 ..."
set -o pipefail
tag=$1; vars=$2
bash tools/gpu_check.sh "$tag" || exit 1
bash tools/ab_variants.sh "gpurun_out/$tag/ab" "$vars $vars" "1"
