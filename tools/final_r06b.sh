#!/bin/bash
# The round-6 record session (tools/final_r06.sh) in two GPU calls that each fit
# gpurun's limit: part a = GPU tests, smoke, the default bench line, its kernel
# trace and PMC passes; part b = C5 on both maps, C3, C4, per-call latencies.
# usage: tools/final_r06b.sh <tag> a|b   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=$1; part=$2; out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
if [ "$part" = a ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -20 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
python tools/bench_brief.py "$out/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err" || { echo "rocprof failed"; tail -20 "$out/rocprof.err"; exit 1; }
python tools/kstats.py "$out/trace/run_kernel_trace.csv" --csv "$out/kernel_stats_by_grid.csv" > "$out/kernel_stats_by_grid.txt"
python tools/kstats.py "$out/trace/run_kernel_trace.csv" --last 10 --csv "$out/kernel_stats_last10.csv" > "$out/kernel_stats_last10.txt"
python tools/overlap.py "$out/trace/run_kernel_trace.csv" --quiet > "$out/overlap.txt"
head -8 "$out/kernel_stats_last10.txt"
bash tools/pmc_profile.sh "$out/pmc" && python tools/pmc_summary.py "$out/pmc" --csv "$out/pmc_summary.csv" > "$out/pmc_summary.txt" || { echo "pmc failed"; exit 1; }
head -6 "$out/pmc_summary.txt"
echo part-a-done
exit 0
fi
timeout -k 10 400 python bench.py --workload c5 > $out/c5_bench.json 2> $out/c5.err || { echo c5 failed; tail -5 $out/c5.err; exit 1; }
python tools/bench_brief.py $out/c5_bench.json
timeout -k 10 400 python bench.py --workload c5 --near-frac 0.1 > $out/c5low_bench.json 2> $out/c5low.err || { echo c5low failed; tail -5 $out/c5low.err; exit 1; }
python tools/bench_brief.py $out/c5low_bench.json
timeout -k 10 300 python bench.py --workload c3 > $out/c3_bench.json 2> $out/c3.err || { echo c3 failed; tail -5 $out/c3.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 > $out/c4_bench.json 2> $out/c4.err || { echo c4 failed; tail -5 $out/c4.err; exit 1; }
python -c "
import json
for w in ('c3', 'c4'):
    d = json.load(open('$out/' + w + '_bench.json')); print(w, d.get('value'), d.get('unit'), d.get('parity'))"
bash tools/gpu_lat.sh $tag 500 - || exit 1
echo alldone

