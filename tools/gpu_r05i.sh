#!/bin/bash
# round 5: in-block LDS grid of the fused projection / initialization searches
set -o pipefail
bash tools/gpu_session.sh r05i "tests=projection or proj or loop or matcher or fisheye or sim3 or fuse or initialization or host_out or bow or streams" || exit 1
bash tools/gpu_lat.sh r05i 200 - 0=4,5=2
