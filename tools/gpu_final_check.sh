#!/bin/bash
# Final-tree check: every GPU test, smoke, one default bench line.
# usage: tools/gpu_final_check.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -20 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
python tools/bench_brief.py "$out/bench.json"
