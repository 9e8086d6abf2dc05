"""Host model of k_sfi_fused's algorithm (tools / CPU tests only).

SearchForInitialization (ORBmatcher.cc:648-763) restated as the fused kernel
computes it: per F1 keypoint of octave 0 the kTopK smallest candidates by
(distance, GetFeaturesInArea order) with distance <= bound, then Jacobi rounds
over every query against the previous round's per-slot claim lists (the skip
rule `vMatchedDistance[i2] <= dist` reads the latest claim on i2 by an earlier
query), exact rescans for truncated lists that cannot decide, and the outputs
from the fixpoint.  `model(...)` returns (nmatches, matches12, prev_out,
rounds, rescans) so tests can compare it with the oracle's serial loop and
see how many rounds the fixpoint took.
"""
from __future__ import annotations

import numpy as np

GRID_COLS, GRID_ROWS, TH_LOW, HISTO, TOPK = 64, 48, 50, 30, 8


def _roundf(v):
    v = np.asarray(v, np.float32)
    return (np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))).astype(np.int64)


def _rot_bin(a1, a2):
    rot = np.float32(a1) - np.float32(a2)
    if rot < 0:
        rot = np.float32(rot + np.float32(360.0))
    b = int(_roundf(np.float32(rot * np.float32(1.0 / HISTO))))
    return 0 if b == HISTO else b


def _three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < 0.1 * m1:
        i2 = i3 = -1
    elif m3 < 0.1 * m1:
        i3 = -1
    return i1, i2, i3


def _candidates(k1, d1, k2, d2, prev, window, grid):
    """Per query: list of (key, d, slot) sorted by key, or None (not a query)."""
    min_x, min_y, inv_w, inv_h = (np.float32(v) for v in grid)
    r = np.float32(window)
    x2, y2 = k2["x"].astype(np.float32), k2["y"].astype(np.float32)
    gx = _roundf((x2 - min_x) * inv_w)
    gy = _roundf((y2 - min_y) * inv_h)
    ingrid = (gx >= 0) & (gx < GRID_COLS) & (gy >= 0) & (gy < GRID_ROWS) & (k2["octave"] == 0)
    bits2 = np.unpackbits(d2, axis=1)
    out = []
    for i in range(len(k1)):
        if k1["octave"][i] != 0:
            out.append(None)
            continue
        px, py = np.float32(prev[i, 0]), np.float32(prev[i, 1])
        x0 = max(0, int(np.floor((px - min_x - r) * inv_w)))
        x1 = min(GRID_COLS - 1, int(np.ceil((px - min_x + r) * inv_w)))
        y0 = max(0, int(np.floor((py - min_y - r) * inv_h)))
        y1 = min(GRID_ROWS - 1, int(np.ceil((py - min_y + r) * inv_h)))
        if x0 >= GRID_COLS or x1 < 0 or y0 >= GRID_ROWS or y1 < 0:
            out.append(None)
            continue
        ok = ingrid & (gx >= x0) & (gx <= x1) & (gy >= y0) & (gy <= y1)
        ok &= (np.abs(x2 - px) < r) & (np.abs(y2 - py) < r)
        idx = np.nonzero(ok)[0]
        dist = (np.unpackbits(d1[i])[None, :] != bits2[idx]).sum(1)
        key = (dist << 24) | ((gx[idx] * GRID_ROWS + gy[idx]) << 12) | idx
        o = np.argsort(key, kind="stable")
        out.append((dist[o].astype(int), idx[o].astype(int)))
    return out


def model(k1, d1, k2, d2, prev, window, ratio, check_ori, grid):
    n1 = len(k1)
    bound = TH_LOW
    while bound < 255 and np.float32(bound + 1) * np.float32(ratio) <= TH_LOW:
        bound += 1
    cands = _candidates(k1, d1, k2, d2, prev, window, grid)
    # phase 1: the lists (entries within the bound) and their counts
    lists, cnt = [], []
    for c in cands:
        if c is None:
            lists.append([])
            cnt.append(-1)
            continue
        dd, ss = c
        keep = dd <= bound
        lists.append(list(zip(dd[keep][:TOPK], ss[keep][:TOPK])))
        cnt.append(int(keep.sum()))

    def accept(best, best2):
        return best <= TH_LOW and np.float32(best) < np.float32(best2) * np.float32(ratio)

    def md_of(claims, s, j):     # latest claim on s before query j
        md = None
        for (jj, d) in claims.get(s, []):
            if jj >= j:
                break
            md = d
        return md

    D = [-2] * n1
    claims = None
    settled = 0
    rounds = rescans = 0
    for rnd in range(n1 + 2):
        rounds += 1
        first_changed = n1
        newD = list(D)
        for j in range(settled, n1):
            c = cnt[j]
            dec = -1
            if c > 0:
                usable = []
                dlast = 0
                for (d, s) in lists[j]:
                    dlast = d
                    if claims is not None:
                        md = md_of(claims, s, j)
                        if md is not None and md <= d:
                            continue
                    usable.append((d, s))
                nav = len(usable)
                exact = c <= TOPK or nav >= 2 or (nav == 1 and (usable[0][0] > TH_LOW or
                                                               np.float32(usable[0][0]) < np.float32(dlast) * np.float32(ratio)))
                if not exact:
                    rescans += 1
                    dd, ss = cands[j]
                    usable = []
                    for d, s in zip(dd, ss):
                        if d > bound:
                            continue
                        md = md_of(claims, s, j)
                        if md is not None and md <= d:
                            continue
                        usable.append((d, s))
                        if len(usable) == 2:
                            break
                if usable:
                    best, slot = usable[0]
                    best2 = usable[1][0] if len(usable) > 1 else 2 ** 31 - 1
                    if accept(best, best2):
                        dec = (slot, best)
            if dec != D[j]:
                first_changed = min(first_changed, j)
            newD[j] = dec
        D = newD
        if first_changed >= n1 and rnd > 0:
            break
        settled = first_changed
        claims = {}
        for j in range(n1):
            if D[j] not in (-1, -2):
                claims.setdefault(D[j][0], []).append((j, D[j][1]))
    # outputs
    last = {s: cl[-1][0] for s, cl in claims.items()}
    hist = [0] * HISTO
    bins = {}
    for j in range(n1):
        if D[j] not in (-1, -2):
            b = _rot_bin(k1["angle"][j], k2["angle"][D[j][0]])
            bins[j] = b
            if check_ori:
                hist[b] += 1
    tm = _three_maxima(hist) if check_ori else (-1, -1, -1)
    m12 = np.full(n1, -1, np.int32)
    nm = len(last)
    for s, j in last.items():
        if check_ori and bins[j] not in tm:
            nm -= 1
        else:
            m12[j] = s
    pout = np.array(prev, np.float32).copy()
    for j in range(n1):
        if m12[j] >= 0:
            pout[j] = (k2["x"][m12[j]], k2["y"][m12[j]])
    return nm, m12, pout, rounds, rescans
