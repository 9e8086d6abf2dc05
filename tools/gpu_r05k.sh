#!/bin/bash
# round 5: fused searches as one launch with a ticket vs two launches
set -o pipefail
bash tools/gpu_session.sh r05k "tests=projection or proj or loop or matcher or initialization or host_out" || exit 1
bash tools/gpu_lat.sh r05k 200 - 0=5,5=3 -
