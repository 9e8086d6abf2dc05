#!/bin/bash
# One GPU validation: the extractor parity suites first (fail fast), then every
# GPU test, then the default bench line.  usage: tools/gpu_check.sh <tag>
set -o pipefail
tag=${1:-chk}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_extractor.py -m gpu > "$out/ext_tests.log" 2>&1 || { echo "extractor tests failed"; tail -40 "$out/ext_tests.log"; exit 1; }
tail -1 "$out/ext_tests.log"
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d["value"]), round(d["ms_per_step"], 3), {k: round(v, 3) for k, v in d["stage_ms"].items() if v})
print("parity", d.get("parity"))
print("roofline", {k: d["roofline"][k] for k in ("frac", "valu_roofline_frac", "ms_per_launch")})
print("north", d["stage_roofline"]["north_star_pyramid_fast_read"]["frac"])
PY
