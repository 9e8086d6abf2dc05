#!/usr/bin/env python3
"""Per-call timing of SearchByProjection(KF, Sim3) (tools/bench_loop.py's
inputs): host wall time per call and the kernels' share via HIP events."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi, orb, synth
    from test_loop_matchers import queries_into
    W, H = 752, 480
    rng = np.random.default_rng(5)
    frames = synth.sequence(W, H, 3, config=9, start=9000)
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    t = ex.tables()
    k, d = ex(frames[1], (0, 0))[:2]
    f = abi.frame_struct(k, d, W, H, scale_factors=t["scale"])
    calls = []
    for _ in range(10):
        va, u, v, lv, de, _, _ = queries_into(k, d, 3000, rng)
        calls.append((f, va, u, v, lv, de, 10, 0.5, np.full(len(k), -1, np.int32)))
    for rep in range(4):
        ts = []
        for c in calls:
            t0 = time.perf_counter()
            orb.ORBmatcher.SearchByProjectionSim3(*c)
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"rep {rep}: " + " ".join(f"{x:.3f}" for x in ts), flush=True)


if __name__ == "__main__":
    main()
