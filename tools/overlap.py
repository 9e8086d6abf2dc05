#!/usr/bin/env python3
"""Stream overlap in a rocprofv3 kernel trace of bench.py (two steps in flight).

For the timed steps (the k_pyr_stream launches of the 256-frame batch, after
the warmup), prints every extraction / matching kernel with its queue, start,
duration and the kernels of OTHER queues it overlaps, then per kernel kind the
share of its time spent beside another queue's kernel and its mean duration in
the timed region vs. the profiled pass (one step in flight, the last 10 of each
kind).  Answers whether step k's latency-bound stages (k_quadtree, k_assemble)
run beside step k+1's k_fast_cells / k_describe, and what that costs each.

usage: tools/overlap.py run_kernel_trace.csv [--steps N] [--quiet]
"""
import argparse
import collections
import csv

KINDS = ("k_pyr_stream", "k_fast_cells", "k_quadtree", "k_describe", "k_assemble", "k_grid_cs", "k_sfi_topk_st",
         "k_sfi_resolve")


def load(path):
    out = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "orbmi::" not in name:
            continue
        kind = name.split("orbmi::")[1].split("(")[0].split("<")[0]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, int(r["Queue_Id"]), grid))
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=6, help="timed steps to analyse (from the 6th batch launch)")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args()
    ks = [k for k in load(a.trace) if k[2] in KINDS]
    big = max(k[4] for k in ks if k[2] == "k_pyr_stream")
    starts = [i for i, k in enumerate(ks) if k[2] == "k_pyr_stream" and k[4] == big]
    i0, i1 = starts[5], starts[min(5 + a.steps, len(starts) - 1)]
    sel = ks[i0:i1]
    base = sel[0][0]
    busy = collections.defaultdict(float)
    beside = collections.defaultdict(float)
    durs = collections.defaultdict(list)
    for s, e, n, q, g in sel:
        others = [o for o in sel if o[3] != q and o[0] < e and o[1] > s]
        # time of [s, e) covered by any other queue's kernel
        iv = sorted((max(s, o[0]), min(e, o[1])) for o in others)
        cov, cur = 0, s
        for x, y in iv:
            if y > cur:
                cov += y - max(x, cur)
                cur = max(cur, y)
        busy[n] += e - s
        beside[n] += cov
        durs[n].append((e - s) / 1000)
        if not a.quiet:
            names = ",".join(sorted({f"{o[2]}@q{o[3]}" for o in others}))
            print(f"{(s - base) / 1000:8.1f} {(e - s) / 1000:7.1f} us q{q} {n:15s} beside: {names}")
    # the profiled pass: the last 10 launches of each kind at the batch grid
    prof = collections.defaultdict(list)
    allk = load(a.trace)
    for n in KINDS:
        g = max((k[4] for k in allk if k[2] == n), default=0)
        xs = [k for k in allk if k[2] == n and k[4] == g]
        prof[n] = [(k[1] - k[0]) / 1000 for k in xs[-10:]]
    span = (sel[-1][1] - base) / 1000
    print(f"\ntimed region: {len(starts[5:5 + a.steps])} steps, {span:.1f} us of kernels")
    print(f"{'kernel':15s} {'beside other queue':>19s} {'mean us timed':>14s} {'mean us alone':>14s}")
    for n in KINDS:
        if busy[n]:
            alone = sum(prof[n]) / max(1, len(prof[n]))
            print(f"{n:15s} {100 * beside[n] / busy[n]:18.0f}% {sum(durs[n]) / len(durs[n]):14.1f} {alone:14.1f}")


if __name__ == "__main__":
    main()
