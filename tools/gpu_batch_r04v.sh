#!/bin/bash
# r04v: k_fast_cells cells per wave (1/2/3/4) and k_describe slots per wave (8/16/32) at the new FAST occupancy.
set -o pipefail
out=gpurun_out/r04v
mkdir -p "$out"
for v in cpw3 ds32; do
  bash tools/variant_tests.sh "$out" $v tests/test_gpu_extractor.py -m gpu || exit 1
done
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "cur cpw1 cpw3 cpw4 ds8 ds32 cur cpw1 cpw3 cpw4 ds8 ds32" || exit 1
