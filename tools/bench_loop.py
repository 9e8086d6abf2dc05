#!/usr/bin/env python3
"""Measurement of the relocalisation / loop-closing matchers
(src/ORBmatcher.cc:427-646,765-905,1340-1674,1889-2010) on synthetic C2
keyframes (752x480, 1000 features), LoopClosing-like sizes:
SearchByBoW(KF1, KF2) of one keyframe against 10 candidates (vocabulary
FeatureVectors, ratio 0.75), SearchByProjection(KF, Sim3) of 3,000 covisible
points (th 10, ratioHamming 0.5), SearchBySim3 of a keyframe pair (th 7.5),
Fuse(KF, Sim3) of 3,000 points into 10 keyframes (th 4), and the
relocalisation SearchByProjection(F, KF) (th 10, ORBdist 100).  GPU host APIs
(per call: upload, grid, kernels, download) vs the CPU oracle on one thread;
parity of every call.
usage: python tools/bench_loop.py"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

W, H = 752, 480


def timed(fn, calls):
    t0 = time.perf_counter()
    out = [fn(*c) for c in calls]
    return out, (time.perf_counter() - t0) / max(1, len(calls)) * 1e3


def same(a, b):
    return all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(a, b))


def main():
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi, orb, synth
    from test_loop_matchers import queries_into, sim3_inputs
    rng = np.random.default_rng(5)
    frames = synth.sequence(W, H, 11, config=9, start=9000)
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    t = ex.tables()
    kfs = [ex(f, (0, 0))[:2] for f in frames]
    voc = abi.vocab_struct(synth.vocabulary(10, 6, seed=31))
    nids = [O.transform(voc, d, 4)[2] for _, d in kfs]
    fs = [abi.frame_struct(k, d, W, H, scale_factors=t["scale"]) for k, d in kfs]
    fvs = [abi.featvec_struct(n) for n in nids]
    valid = [(rng.random(len(k)) < 0.7).astype(np.uint8) for k, _ in kfs]
    m = orb.ORBmatcher(0.75, True)
    res = {}

    calls = [(fs[0], fvs[0], valid[0], fs[j], fvs[j], valid[j]) for j in range(1, 11)]
    m.SearchByBoWKF(*calls[0])
    g, tg = timed(m.SearchByBoWKF, calls)
    r, tc = timed(lambda *c: O.search_by_bow_kf(*c, 0.75, True), calls)
    res["search_by_bow_kf"] = {"calls": len(calls), "gpu_ms_per_call": tg, "cpu_ms_per_call": tc,
                               "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                               "mean_matches": float(np.mean([x[0] for x in g]))}

    k, d = kfs[1]
    calls = []
    for _ in range(10):
        va, u, v, lv, de, _, _ = queries_into(k, d, 3000, rng)
        calls.append((fs[1], va, u, v, lv, de, 10, 0.5, np.full(len(k), -1, np.int32)))
    orb.ORBmatcher.SearchByProjectionSim3(*calls[0])
    g, tg = timed(orb.ORBmatcher.SearchByProjectionSim3, calls)
    r, tc = timed(O.search_by_projection_sim3, calls)
    res["search_by_projection_sim3"] = {"calls": len(calls), "points_per_call": 3000, "gpu_ms_per_call": tg,
                                        "cpu_ms_per_call": tc,
                                        "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                                        "mean_matches": float(np.mean([x[0] for x in g]))}

    calls = []
    for j in range(1, 11):
        _, _, _, _, q1, q2 = sim3_inputs(([kfs[0], kfs[j]], t), 20 + j)
        calls.append((fs[0], fs[j], q1, q2, 7.5))
    orb.ORBmatcher.SearchBySim3(*calls[0])
    g, tg = timed(orb.ORBmatcher.SearchBySim3, calls)
    r, tc = timed(O.search_by_sim3, calls)
    res["search_by_sim3"] = {"calls": len(calls), "gpu_ms_per_call": tg, "cpu_ms_per_call": tc,
                             "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                             "mean_found": float(np.mean([x[0] for x in g]))}

    calls = []
    for j in range(1, 11):
        k, d = kfs[j]
        va, u, v, lv, de, _, _ = queries_into(k, d, 3000, rng)
        calls.append((fs[j], va, u, v, lv, de, 4.0))
    orb.ORBmatcher.FuseSim3(*calls[0])
    g, tg = timed(orb.ORBmatcher.FuseSim3, calls)
    r, tc = timed(O.fuse_sim3, calls)
    res["fuse_sim3"] = {"calls": len(calls), "points_per_call": 3000, "gpu_ms_per_call": tg, "cpu_ms_per_call": tc,
                        "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                        "mean_fused": float(np.mean([x[0] for x in g]))}

    calls = []
    for j in range(1, 11):
        k, d = kfs[j]
        va, u, v, lv, de, ang, _ = queries_into(k, d, 1000, rng)
        calls.append((fs[j], va, u, v, lv, ang, de, 10, 100, np.full(len(k), -1, np.int32)))
    m.SearchByProjectionKF(*calls[0])
    g, tg = timed(m.SearchByProjectionKF, calls)
    r, tc = timed(lambda *c: O.search_by_projection_kf(*c[:9], True, c[9]), calls)
    res["search_by_projection_kf"] = {"calls": len(calls), "points_per_call": 1000, "gpu_ms_per_call": tg,
                                      "cpu_ms_per_call": tc,
                                      "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                                      "mean_matches": float(np.mean([x[0] for x in g]))}
    # tracking: SearchByProjection(F, local map points) (TrackLocalMap, th 3) and
    # SearchByProjection(F, LastFrame) (TrackWithMotionModel, th 7 at mode 0)
    calls, calls_last = [], []
    for j in range(1, 11):
        k, d = kfs[j]
        n = 3000
        src = rng.integers(0, len(k), n)
        qx = (k["x"][src] + rng.normal(0, 2, n)).astype(np.float32)
        qy = (k["y"][src] + rng.normal(0, 2, n)).astype(np.float32)
        lvl = np.clip(k["octave"][src] + rng.integers(0, 2, n), 0, 7).astype(np.int32)
        qd = d[src].copy()
        qd[rng.random((n, 32)) < 0.03] ^= np.uint8(0x10)
        mps = abi.mappoints_struct(qx, qy, qx - 20, lvl, rng.uniform(0.99, 1.0, n).astype(np.float32),
                                   rng.uniform(0, 100, n).astype(np.float32), (rng.random(n) < 0.9).astype(np.uint8),
                                   (rng.random(n) < 0.7).astype(np.uint8), qd)
        owner = np.full(len(k), -1, np.int32)
        calls.append((fs[j], mps, owner))
        nl = 1000
        sl = src[:nl]
        calls_last.append((fs[j], (rng.random(nl) < 0.9).astype(np.uint8), qx[:nl], qy[:nl], (qx[:nl] - 20),
                           k["octave"][sl].astype(np.int32), k["angle"][sl], (rng.random(nl) < 0.7).astype(np.uint8),
                           qd[:nl], 7.0, 0))
    mp = orb.ORBmatcher(0.8, True)
    f_mps = lambda F, mps, owner: mp.SearchByProjection(F, mps, 3.0, False, 50.0, owner, None)
    r_mps = lambda F, mps, owner: O.search_by_projection_mps(F, mps, 3.0, False, 50.0, 0.8, owner,
                                                             np.zeros(F.struct.n, np.uint8))
    f_mps(*calls[0])
    g, tg = timed(f_mps, calls)
    r, tc = timed(r_mps, calls)
    res["search_by_projection_mps"] = {"calls": len(calls), "points_per_call": 3000, "gpu_ms_per_call": tg,
                                       "cpu_ms_per_call": tc,
                                       "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                                       "mean_matches": float(np.mean([x[0] for x in g]))}
    ml = orb.ORBmatcher(0.9, True)
    zero = lambda F: (np.full(F.struct.n, -1, np.int32), np.zeros(F.struct.n, np.uint8))
    f_last = lambda F, *q: ml.SearchByProjectionLast(F, *q, owner=zero(F)[0], blocked=zero(F)[1])
    r_last = lambda F, *q: O.search_by_projection_last(F, *q, True, *zero(F))
    f_last(*calls_last[0])
    g, tg = timed(f_last, calls_last)
    r, tc = timed(r_last, calls_last)
    res["search_by_projection_last"] = {"calls": len(calls_last), "points_per_call": 1000, "gpu_ms_per_call": tg,
                                        "cpu_ms_per_call": tc,
                                        "mismatched": sum(int(not same(x, y)) for x, y in zip(g, r)),
                                        "mean_matches": float(np.mean([x[0] for x in g]))}

    # relocalisation: SearchByBoW(KF_i, F) over 10 candidates (Tracking.cc:3641-3648)
    # as one orbm_search_by_bow_many call vs the oracle looping over them
    cand = list(range(1, 11))
    mm = orb.ORBmatcher(0.75, True)
    args = ([fs[j] for j in cand], [fvs[j] for j in cand], [valid[j] for j in cand], fs[0], fvs[0])
    mm.SearchByBoWMany(*args)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        gc, gmatch = mm.SearchByBoWMany(*args)
    tg = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        rr = [O.search_by_bow(fs[j], fvs[j], valid[j], fs[0], fvs[0], 0.75, True) for j in cand]
    tc = (time.perf_counter() - t0) / reps * 1e3
    bad = sum(int(gc[i] != rr[i][0] or not np.array_equal(gmatch[i], rr[i][1])) for i in range(len(cand)))
    res["search_by_bow_many"] = {"calls": reps, "candidates_per_call": len(cand), "gpu_ms_per_call": tg,
                                 "cpu_ms_per_call": tc, "mismatched": bad, "mean_matches": float(np.mean(gc))}
    print(json.dumps({"metric": "tracking / relocalisation / loop-closing matchers, host APIs", "n_gpus": 1,
                      "data": "synthetic", "cpu_baseline_kind": "port, 1 thread", "results": res}), flush=True)


if __name__ == "__main__":
    main()
