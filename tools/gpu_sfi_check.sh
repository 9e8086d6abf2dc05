#!/bin/bash
# SearchForInitialization GPU check: the matcher GPU tests, then the
# k_sfi_resolve A/B of variants and the walk phase probe.
# usage: tools/gpu_sfi_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/sfi_check}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_dframe.py tests/test_gpu_host_out.py tests/test_gpu_streams.py tests/test_gpu_cpp_api.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_sfi_ab.sh $OUT/ab "${2:-sfidef qst sfidef qst}" && bash tools/gpu_sfi_probe.sh $OUT/probe
