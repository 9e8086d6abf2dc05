#!/bin/bash
# One parameterised GPU session (replaces the per-batch one-off scripts).
# usage: tools/gpu_session.sh <tag> <step> [<step> ...]   outputs under gpurun_out/<tag>/
# steps (run in order; the first failure ends the session, nothing after it runs):
#   tests[=<pytest -k expr>]      GPU tests (all of them without an expression)
#   smoke                         __graft_entry__.smoke()
#   bench[=<bench.py args>]       one bench line -> bench_<i>.json
#   trace[=<bench.py args>]       rocprofv3 --kernel-trace --stats of bench.py -> trace_<i>/, kstats_<i>.txt
#                                 (all launches) and kstats_last_<i>.txt (the profiled pass: last 10 per grid)
#   pmc[=<bench.py args>]         tools/pmc_profile.sh passes -> pmc_<i>/ + pmc_summary_<i>.csv
#   py=<script and args>          python -u <script and args> -> py_<i>.log
#   lib=<path to a prebuilt .so>  swap the product library for the following steps (restored at the end)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
LIB=orb_slam3_vio_fixes_amd/liborb_mi355x.so
cp "$LIB" "$out/.default.so"
restore() { cp "$out/.default.so" "$LIB"; }
trap restore EXIT
i=0
for st in "$@"; do
  i=$((i+1)); name=${st%%=*}; arg=""; [[ $st == *=* ]] && arg=${st#*=}
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${k[@]}" > "$out/tests_$i.log" 2>&1 \
        || { echo "[$i] tests failed"; tail -30 "$out/tests_$i.log"; exit 1; }
      tail -1 "$out/tests_$i.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke_$i.log" 2>&1 \
        || { echo "[$i] smoke failed"; tail -20 "$out/smoke_$i.log"; exit 1; }
      tail -1 "$out/smoke_$i.log" ;;
    bench)
      timeout -k 10 600 python bench.py $arg > "$out/bench_$i.json" 2> "$out/bench_$i.err" \
        || { echo "[$i] bench failed"; tail -20 "$out/bench_$i.err"; exit 1; }
      python tools/bench_brief.py "$out/bench_$i.json" ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_$i" -o run -- python3 bench.py $arg \
        > "$out/trace_$i.json" 2> "$out/trace_$i.err" || { echo "[$i] trace failed"; tail -20 "$out/trace_$i.err"; exit 1; }
      python tools/kstats.py "$out/trace_$i/run_kernel_trace.csv" --csv "$out/kstats_$i.csv" > "$out/kstats_$i.txt"
      python tools/kstats.py "$out/trace_$i/run_kernel_trace.csv" --last 10 --csv "$out/kstats_last_$i.csv" > "$out/kstats_last_$i.txt"
      head -8 "$out/kstats_last_$i.txt" ;;
    pmc)
      a=${arg:---steps 3 --warmup 1 --cpu-sample 0 --no-host-api --no-profile --overlap 1 --sets 2}
      bash tools/pmc_profile.sh "$out/pmc_$i" $a || { echo "[$i] pmc failed"; exit 1; }
      python tools/pmc_summary.py "$out/pmc_$i" --csv "$out/pmc_summary_$i.csv" > "$out/pmc_summary_$i.txt"
      head -12 "$out/pmc_summary_$i.txt" ;;
    py)
      timeout -k 10 600 python -u $arg > "$out/py_$i.log" 2>&1 || { echo "[$i] py failed"; tail -20 "$out/py_$i.log"; exit 1; }
      tail -5 "$out/py_$i.log" ;;
    lib)
      cp "$arg" "$LIB" || exit 1
      echo "[$i] library: $arg" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "session $tag done"
