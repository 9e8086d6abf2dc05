#!/usr/bin/env python3
"""Measurement of SURVEY.md §8(f) row 3: DetectRelocalizationCandidates over a
synthetic 10,000-keyframe database (vocabulary of 10^5 words, 80-300 words
per keyframe, Zipf-like word frequencies), GPU path (orbk_*) vs the CPU
oracle, queries/s and the parity of every query.
usage: python tools/bench_reloc.py [--nkf 10000] [--queries 50]"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nkf", type=int, default=10000)
    ap.add_argument("--nwords", type=int, default=100000)
    ap.add_argument("--queries", type=int, default=50)
    args = ap.parse_args()
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import orb
    from tests import kfdb_ref as R
    db = R.make_db(args.nkf, args.nwords, 11)
    qs = [R.make_query(db, 1000 + i) for i in range(args.queries)]
    gdb = orb.KeyFrameDatabase(db)
    a = np.zeros(args.nkf, np.float32)
    b = a.copy()
    gdb.DetectRelocalizationCandidates(*qs[0], 0, a.copy())        # warm-up
    t0 = time.perf_counter()
    got = [gdb.DetectRelocalizationCandidates(qw, qv, i % 2, a) for i, (qw, qv) in enumerate(qs)]
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref = [O.detect_relocalization_candidates(db, qw, qv, i % 2, b) for i, (qw, qv) in enumerate(qs)]
    tc = time.perf_counter() - t0
    bad = sum(list(x) != list(y) for x, y in zip(got, ref)) + int(not np.array_equal(a, b))
    print(json.dumps({"metric": "relocalization queries/s (DetectRelocalizationCandidates, 10k-KF database)",
                      "value": args.queries / tg, "unit": "queries/s", "n_gpus": 1, "higher_is_better": True,
                      "config": {"workload": f"{args.nkf} keyframes, {args.nwords} words, synthetic BowVectors",
                                 "queries": args.queries},
                      "ms_per_query": tg / args.queries * 1e3,
                      "cpu_baseline": {"value": args.queries / tc, "unit": "queries/s", "cores": 1, "kind": "port",
                                       "sample": "the same queries through the oracle"},
                      "parity": {"queries_checked": args.queries, "mismatched": bad},
                      "mean_candidates": float(np.mean([len(x) for x in got]))}), flush=True)


if __name__ == "__main__":
    main()
