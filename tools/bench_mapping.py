#!/usr/bin/env python3
"""Measurement of SURVEY.md §8(f) row 4 (mapping-thread matchers), one
LocalMapping-like round on synthetic C2 keyframes (752x480, 1000 features):
SearchForTriangulation of one keyframe against 10 neighbours, Fuse of 3,000
map points into 10 keyframes, ComputeDistinctiveDescriptors for 5,000 points
with 2-30 observations.  GPU host APIs vs the CPU oracle; parity of every call.
usage: python tools/bench_mapping.py"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

W, H = 752, 480


def main():
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi, orb, synth
    from tests.test_mapping import F12_and_ep
    rng = np.random.default_rng(3)
    frames = synth.sequence(W, H, 11, config=2, start=7000)
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    t = ex.tables()
    kfs = [ex(f, (0, 0))[:2] for f in frames]
    voc = abi.vocab_struct(synth.vocabulary(10, 6, seed=31))
    nids = [O.transform(voc, d, 4)[2] for _, d in kfs]
    F, ep = F12_and_ep()
    frames_s = [abi.frame_struct(k, d, W, H, scale_factors=t["scale"]) for k, d in kfs]
    fvs = [abi.featvec_struct(n) for n in nids]
    mps = [(rng.random(len(k)) < 0.3).astype(np.uint8) for k, _ in kfs]
    m = orb.ORBmatcher(0.6, True)
    res = {}
    # SearchForTriangulation: KF 0 against KFs 1..10
    calls = [(0, j) for j in range(1, 11)]
    m.SearchForTriangulation(frames_s[0], fvs[0], mps[0], frames_s[1], fvs[1], mps[1], F, ep, t["sigma2"])
    t0 = time.perf_counter()
    g = [m.SearchForTriangulation(frames_s[a], fvs[a], mps[a], frames_s[b], fvs[b], mps[b], F, ep, t["sigma2"])
         for a, b in calls]
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    r = [O.search_for_triangulation(frames_s[a], fvs[a], mps[a], frames_s[b], fvs[b], mps[b], F, ep, t["sigma2"])
         for a, b in calls]
    tc = time.perf_counter() - t0
    res["search_for_triangulation"] = {"calls": len(calls), "gpu_ms_per_call": tg / len(calls) * 1e3,
                                       "cpu_ms_per_call": tc / len(calls) * 1e3,
                                       "mismatched": sum(int(x[0] != y[0] or not np.array_equal(x[1], y[1]))
                                                         for x, y in zip(g, r)),
                                       "mean_matches": float(np.mean([x[0] for x in g]))}
    # Fuse: 3,000 points into each of 10 keyframes
    npt = 3000
    gf, rf = [], []
    tg = tc = 0.0
    for j in range(1, 11):
        k, d = kfs[j]
        sel = rng.integers(0, len(k), npt)
        u = (k["x"][sel] + rng.normal(0, 2, npt)).astype(np.float32)
        v = (k["y"][sel] + rng.normal(0, 2, npt)).astype(np.float32)
        lvl = np.minimum(k["octave"][sel] + rng.integers(0, 2, npt), 7).astype(np.int32)
        bits = np.unpackbits(d[sel], axis=1)
        md = np.packbits(bits ^ (rng.random(bits.shape) < 0.06), axis=1)
        valid = (rng.random(npt) < 0.9).astype(np.uint8)
        ur = u.copy()
        t0 = time.perf_counter()
        gf.append(orb.ORBmatcher.Fuse(frames_s[j], t["inv_sigma2"], valid, u, v, ur, lvl, md, 3.0))
        tg += time.perf_counter() - t0
        t0 = time.perf_counter()
        rf.append(O.fuse(frames_s[j], t["inv_sigma2"], valid, u, v, ur, lvl, md, 3.0))
        tc += time.perf_counter() - t0
    res["fuse"] = {"calls": 10, "points_per_call": npt, "gpu_ms_per_call": tg / 10 * 1e3,
                   "cpu_ms_per_call": tc / 10 * 1e3,
                   "mismatched": sum(int(not np.array_equal(x[1], y[1])) for x, y in zip(gf, rf)),
                   "mean_fused": float(np.mean([x[0] for x in gf]))}
    # ComputeDistinctiveDescriptors: 5,000 points
    sizes = rng.integers(2, 31, 5000)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    desc = rng.integers(0, 256, (off[-1], 32), dtype=np.uint8)
    orb.compute_distinctive_descriptors(off[:11], desc)
    t0 = time.perf_counter()
    gb = orb.compute_distinctive_descriptors(off, desc)
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    rb = O.compute_distinctive_descriptors(off, desc)
    tc = time.perf_counter() - t0
    res["compute_distinctive_descriptors"] = {"points": 5000, "gpu_ms": tg * 1e3, "cpu_ms": tc * 1e3,
                                              "mismatched": int((gb != rb).sum())}
    print(json.dumps({"metric": "mapping matchers (SURVEY §8(f) row 4), host APIs", "n_gpus": 1,
                      "data": "synthetic", "cpu_baseline_kind": "port, 1 thread", "results": res}), flush=True)


if __name__ == "__main__":
    main()
