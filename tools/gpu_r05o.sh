#!/bin/bash
# host-call uploads by a pull kernel vs hipMemcpyAsync: GPU tests of the host APIs + latency A/B
set -o pipefail
bash tools/gpu_session.sh r05o "tests=matcher or proj or loop or fisheye or sim3 or fuse or initialization or host_out or bow or mapping or stereo or vocab or kfdb or cpp_api or adapter or streams" || exit 1
bash tools/gpu_lat.sh r05o 200 - 6=1 6=2 -
