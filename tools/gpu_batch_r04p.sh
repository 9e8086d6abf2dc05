#!/bin/bash
# r04p: k_fast_cells occupancy probe: extra LDS per block (4 -> 3 waves a SIMD at +3000 B).
set -o pipefail
out=gpurun_out/r04p
mkdir -p "$out"
NOPMC=1 bash tools/prof_variants.sh "$out/prof" "p0 p2 p3 p0 p2 p3" || exit 1
