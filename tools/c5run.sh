set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py --workload c5 --cpu-sample 20 > $out/c5.json 2> $out/c5.err || { echo bench failed; tail -20 $out/c5.err; exit 1; }
python -c "import json; d=json.load(open('$out/c5.json')); print(d['ms_per_query'], d['parity'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --workload c5 --cpu-sample 0 > $out/c5_prof.json 2> $out/prof.err || { echo prof failed; tail -20 $out/prof.err; exit 1; }
python tools/kstats.py $out/trace/run_kernel_trace.csv > $out/kstats.txt; head -12 $out/kstats.txt
