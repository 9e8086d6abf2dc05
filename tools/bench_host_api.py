#!/usr/bin/env python3
"""PCIe-inclusive rates of the host-buffer extractor APIs (the drop-in path a
Tracking thread calls with a cv::Mat): orbx_extract on one 752x480 image per
call (upload, pipeline, download: latency) and orbx_extract_batch on B host
images per call.  Not the headline metric (bench.py keeps inputs resident in
HBM); reported in DESIGN.md.  usage: python tools/bench_host_api.py"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from orb_slam3_vio_fixes_amd import orb, synth
    imgs = synth.sequence(752, 480, 64, config=2, start=700)
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    res = {}
    for _ in range(3):
        ex(imgs[0], None, (0, 1000))
    n = 50
    t0 = time.perf_counter()
    for i in range(n):
        ex(imgs[i % len(imgs)], None, (0, 1000))
    dt = (time.perf_counter() - t0) / n
    res["orbx_extract_1_image"] = {"ms_per_call": dt * 1e3, "frames_per_s": 1 / dt}
    for B in (2, 16, 64):
        batch = list(imgs[:B])
        ex.extract_batch(batch)
        reps = max(3, 64 // B)
        t0 = time.perf_counter()
        for _ in range(reps):
            ex.extract_batch(batch)
        dt = (time.perf_counter() - t0) / reps
        res[f"orbx_extract_batch_{B}_images"] = {"ms_per_call": dt * 1e3, "frames_per_s": B / dt}
    print(json.dumps({"metric": "host-buffer extraction, PCIe-inclusive (752x480, 1000 features)", "n_gpus": 1,
                      "data": "synthetic", "results": res}), flush=True)


if __name__ == "__main__":
    main()
