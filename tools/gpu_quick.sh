#!/bin/bash
# Quick GPU iteration: a test selection, then the default bench without the CPU
# legs, then a kernel-trace of the same bench.  usage: tools/gpu_quick.sh <tag> "<pytest -k expr>"
set -o pipefail
tag=${1:-quick}; sel=${2:-pyramid}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$sel" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 300 python bench.py --cpu-sample 0 --no-host-api > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$out/bench.json')); print(round(d['value']), {k: round(v*1e3,1) for k,v in d['stage_ms'].items() if v})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --cpu-sample 0 --no-host-api > "$out/bench_prof.json" 2> "$out/prof.err" || { echo "rocprof failed"; tail -20 "$out/prof.err"; exit 1; }
python tools/kstats.py "$out/trace/run_kernel_trace.csv" | head -12
