#!/bin/bash
# extraction host call with the pull-kernel upload: host-API tests + the bench's host_api block
set -o pipefail
bash tools/gpu_session.sh r05p "tests=extractor or adapter or cpp_api or configs or host or smoke" "bench=--cpu-sample 0" || exit 1
python -c "
import json
d = json.loads(open('gpurun_out/r05p/bench_2.json').read().strip().splitlines()[-1])
h = d['host_api']; print({k: v for k, v in h.items() if k != 'matchers'})
print({k: v['median_us'] for k, v in h['matchers']['gpu'].items() if 'median_us' in v})"
