#!/bin/bash
# C5 top-4: skip empty rows of partial tiles (A/B against the previous build) + C5 tests
set -o pipefail
bash tools/gpu_session.sh r05n "tests=c5" || exit 1
bash tools/ab_c5.sh gpurun_out/r05n/ab "c5base c5skip c5base c5skip"
