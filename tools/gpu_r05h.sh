#!/bin/bash
set -o pipefail
B="--cpu-sample 0 --no-host-api"
D=orb_slam3_vio_fixes_amd/.r05h_default.so
bash tools/gpu_session.sh r05h "tests=projection or proj or loop or matcher or fisheye or sim3 or fuse or extractor or configs or fast or bow or initialization or host_out" \
  "bench=$B" "lib=variants/lib_inc0.so" "bench=$B" "lib=variants/lib_celloff0.so" "bench=$B" \
  "lib=$D" "bench=$B" "lib=variants/lib_inc0.so" "bench=$B" "lib=variants/lib_celloff0.so" "bench=$B" || exit 1
cp $D orb_slam3_vio_fixes_amd/liborb_mi355x.so
bash tools/gpu_lat.sh r05h 200 - 6=1 5=1 5=1,6=1
