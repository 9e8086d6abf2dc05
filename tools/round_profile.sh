#!/bin/bash
# One GPU session: GPU tests, the default bench line, a rocprofv3 kernel-trace
# --stats run of the same bench command, and the PMC passes.
# usage: tools/round_profile.sh <tag>      (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-prof}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -20 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err" || { echo "rocprof failed"; tail -20 "$out/rocprof.err"; exit 1; }
python tools/kstats.py "$out/trace/run_kernel_trace.csv" --csv "$out/kernel_stats_by_grid.csv" > "$out/kernel_stats_by_grid.txt"
tools/pmc_profile.sh "$out/pmc" && python tools/pmc_summary.py "$out/pmc" --csv "$out/pmc_summary.csv" > "$out/pmc_summary.txt"
echo done
