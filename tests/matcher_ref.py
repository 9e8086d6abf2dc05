"""Independent pure-Python restatements of the matcher semantics (small
inputs only), used to cross-check the C++ oracle.  Reference lines:
Frame.cc:657-735 (grid), ORBmatcher.cc:648-763 (SearchForInitialization),
:223-425 (SearchByBoW), :43-213 (SearchByProjection, map points),
:1676-1887 (SearchByProjection, last frame), :2012-2074."""
import math

import numpy as np

TH_HIGH, TH_LOW, HISTO = 100, 50, 30
f32 = np.float32


def hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def grid(kps, w, h):
    inv_w, inv_h = f32(64) / f32(w), f32(48) / f32(h)
    cells = {}
    for i, k in enumerate(kps):
        gx = int(np.round(f32(f32(k["x"]) - f32(0)) * inv_w))
        gy = int(np.round(f32(f32(k["y"]) - f32(0)) * inv_h))
        # std::round is half away from zero; np.round is half-even: fix ties
        vx, vy = f32(f32(k["x"]) * inv_w), f32(f32(k["y"]) * inv_h)
        gx = int(math.floor(float(vx) + 0.5)) if vx >= 0 else -int(math.floor(-float(vx) + 0.5))
        gy = int(math.floor(float(vy) + 0.5)) if vy >= 0 else -int(math.floor(-float(vy) + 0.5))
        if 0 <= gx < 64 and 0 <= gy < 48:
            cells.setdefault((gx, gy), []).append(i)
    return cells, inv_w, inv_h


def area(kps, g, x, y, r, minL=-1, maxL=-1):
    cells, iw, ih = g
    x, y, r = f32(x), f32(y), f32(r)
    cx0 = max(0, int(math.floor(f32(f32(x - f32(0)) - r) * iw)))
    if cx0 >= 64:
        return []
    cx1 = min(63, int(math.ceil(f32(f32(x - f32(0)) + r) * iw)))
    if cx1 < 0:
        return []
    cy0 = max(0, int(math.floor(f32(f32(y - f32(0)) - r) * ih)))
    if cy0 >= 48:
        return []
    cy1 = min(47, int(math.ceil(f32(f32(y - f32(0)) + r) * ih)))
    if cy1 < 0:
        return []
    chk = minL > 0 or maxL >= 0
    out = []
    for ix in range(cx0, cx1 + 1):
        for iy in range(cy0, cy1 + 1):
            for i in cells.get((ix, iy), []):
                k = kps[i]
                if chk and (k["octave"] < minL or (maxL >= 0 and k["octave"] > maxL)):
                    continue
                if abs(f32(k["x"]) - x) < r and abs(f32(k["y"]) - y) < r:
                    out.append(i)
    return out


def rot_bin(a1, a2):
    rot = f32(f32(a1) - f32(a2))
    if rot < 0:
        rot = f32(rot + f32(360))
    v = float(f32(rot * f32(1.0 / 30)))
    b = int(math.floor(v + 0.5))
    return 0 if b == HISTO else b


def three_maxima(sizes):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(sizes):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def search_for_initialization(k1, d1, k2, d2, w, h, prev, window, ratio, check_ori):
    g2 = grid(k2, w, h)
    m12 = [-1] * len(k1)
    mdist = [2 ** 31 - 1] * len(k2)
    m21 = [-1] * len(k2)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i1 in range(len(k1)):
        if k1[i1]["octave"] > 0:
            continue
        cand = area(k2, g2, prev[i1][0], prev[i1][1], window, k1[i1]["octave"], k1[i1]["octave"])
        if not cand:
            continue
        best = best2 = 2 ** 31 - 1
        bi = -1
        for i2 in cand:
            dist = hamming(d1[i1], d2[i2])
            if mdist[i2] <= dist:
                continue
            if dist < best:
                best2, best, bi = best, dist, i2
            elif dist < best2:
                best2 = dist
        if best <= TH_LOW and f32(best) < f32(f32(best2) * f32(ratio)):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1], m21[bi], mdist[bi] = bi, i1, best
            nm += 1
            if check_ori:
                hist[rot_bin(k1[i1]["angle"], k2[bi]["angle"])].append(i1)
    if check_ori:
        keep = three_maxima([len(x) for x in hist])
        for b in range(HISTO):
            if b in keep:
                continue
            for i1 in hist[b]:
                if m12[i1] >= 0:
                    m12[i1] = -1
                    nm -= 1
    return nm, np.array(m12, np.int32)


def search_by_bow(kk, kd, kfv, kvalid, fk, fd, ffv, ratio, check_ori):
    """kfv/ffv: dict node -> list of feature indices."""
    match = [-1] * len(fk)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for node in sorted(set(kfv) & set(ffv)):
        for ikf in kfv[node]:
            if not kvalid[ikf]:
                continue
            best = best2 = 256
            bi = -1
            for jf in ffv[node]:
                if match[jf] >= 0:
                    continue
                dist = hamming(kd[ikf], fd[jf])
                if dist < best:
                    best2, best, bi = best, dist, jf
                elif dist < best2:
                    best2 = dist
            if best <= TH_LOW and f32(best) < f32(f32(ratio) * f32(best2)):
                match[bi] = ikf
                if check_ori:
                    hist[rot_bin(kk[ikf]["angle"], fk[bi]["angle"])].append(bi)
                nm += 1
    if check_ori:
        keep = three_maxima([len(x) for x in hist])
        for b in range(HISTO):
            if b in keep:
                continue
            for j in hist[b]:
                match[j] = -1
                nm -= 1
    return nm, np.array(match, np.int32)
