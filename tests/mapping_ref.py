"""Independent Python restatements of the mapping-thread matchers
(ORBmatcher::Fuse(pKF, vpMapPoints, th), src/ORBmatcher.cc:1148-1331, and
ORBmatcher::SearchForTriangulation, :907-1146, with
Pinhole::epipolarConstrain, Pinhole.cpp:107-129) used to pin the C++ oracle.
float32 arithmetic throughout; fused multiply-adds are evaluated exactly
(rational arithmetic, one rounding to float32)."""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

f32 = np.float32
TH_LOW, HISTO = 50, 30


def _round_f32(x: Fraction) -> np.float32:
    if x == 0:
        return f32(0.0)
    s = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    # x in [2^e, 2^(e+1)): 24-bit significand
    scaled = x / (Fraction(2) ** (e - 23))
    n = scaled.numerator // scaled.denominator
    rem = scaled - n
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
        n += 1
    return f32(s * math.ldexp(float(n), e - 23))


def fmaf(a, b, c) -> np.float32:
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def sq2(a, b, fma):
    return fmaf(a, a, f32(b) * f32(b)) if fma else f32(f32(a) * f32(a) + f32(b) * f32(b))


def lin2(x, a, y, b, c, fma):
    if fma:
        return f32(fmaf(x, a, f32(y) * f32(b)) + f32(c))
    return f32(f32(f32(x) * f32(a) + f32(y) * f32(b)) + f32(c))


def area(kps, grid, x, y, r):
    """KeyFrame::GetFeaturesInArea (KeyFrame.cc:704-748): ix outer, iy inner,
    cell lists in index order."""
    min_x, min_y, inv_w, inv_h, cells = grid
    x0 = max(0, int(math.floor(f32(f32(f32(x) - min_x) - r) * inv_w)))
    if x0 >= 64:
        return []
    x1 = min(63, int(math.ceil(f32(f32(f32(x) - min_x) + r) * inv_w)))
    if x1 < 0:
        return []
    y0 = max(0, int(math.floor(f32(f32(f32(y) - min_y) - r) * inv_h)))
    if y0 >= 48:
        return []
    y1 = min(47, int(math.ceil(f32(f32(f32(y) - min_y) + r) * inv_h)))
    if y1 < 0:
        return []
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in cells.get((ix, iy), []):
                if abs(f32(kps["x"][i] - f32(x))) < r and abs(f32(kps["y"][i] - f32(y))) < r:
                    out.append(i)
    return out


def _round_away(x) -> int:
    return int(math.floor(float(x) + 0.5)) if x >= 0 else -int(math.floor(-float(x) + 0.5))


def make_grid(kps, min_x, max_x, min_y, max_y):
    inv_w = f32(f32(64) / f32(max_x - min_x))
    inv_h = f32(f32(48) / f32(max_y - min_y))
    cells = {}
    for i in range(len(kps)):
        gx = _round_away(f32(f32(kps["x"][i] - f32(min_x)) * inv_w))
        gy = _round_away(f32(f32(kps["y"][i] - f32(min_y)) * inv_h))
        if 0 <= gx < 64 and 0 <= gy < 48:
            cells.setdefault((gx, gy), []).append(i)
    return (f32(min_x), f32(min_y), inv_w, inv_h, cells)


def fuse(kps, desc, u_right, scale, inv_sigma2, grid, valid, u, v, ur, level, mdesc, th, fma=1):
    n = len(valid)
    bi = np.full(n, -1, np.int32)
    for i in range(n):
        if not valid[i]:
            continue
        pl = int(level[i])
        r = f32(f32(th) * scale[pl])
        cand = area(kps, grid, u[i], v[i], r)
        best, bidx = 256, -1
        for idx in cand:
            kl = int(kps["octave"][idx])
            if kl < pl - 1 or kl > pl:
                continue
            ex, ey = f32(u[i] - kps["x"][idx]), f32(v[i] - kps["y"][idx])
            if u_right is not None and u_right[idx] >= 0:
                er = f32(ur[i] - u_right[idx])
                e2 = fmaf(er, er, fmaf(ex, ex, f32(ey * ey))) if fma else f32(f32(ex * ex + ey * ey) + er * er)
                if float(f32(e2 * inv_sigma2[kl])) > 7.8:
                    continue
            else:
                e2 = sq2(ex, ey, fma)
                if float(f32(e2 * inv_sigma2[kl])) > 5.99:
                    continue
            d = int(np.unpackbits(np.bitwise_xor(mdesc[i], desc[idx])).sum())
            if d < best:
                best, bidx = d, idx
        if best <= TH_LOW:
            bi[i] = bidx
    return bi


def rot_bin(a1, a2):
    rot = f32(f32(a1) - f32(a2))
    if rot < 0.0:
        rot = f32(rot + f32(360.0))
    x = f32(rot * f32(1.0 / 30))
    b = int(math.floor(float(x) + 0.5))
    return 0 if b == HISTO else b


def three_maxima(counts):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(counts):
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


def search_for_triangulation(k1, d1, ur1, mp1, fv1, k2, d2, ur2, mp2, fv2, scale2, sigma2_2, F, ep, only_stereo,
                             coarse, check_ori, fma=1):
    F = np.asarray(F, np.float32).reshape(9)
    m12 = np.full(len(k1), -1, np.int32)
    hist = [[] for _ in range(HISTO)]
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if mp1[i1]:
                continue
            st1 = ur1 is not None and ur1[i1] >= 0
            if only_stereo and not st1:
                continue
            best_d, best = TH_LOW, -1
            for i2 in fv2[node]:
                if mp2[i2]:
                    continue
                st2 = ur2 is not None and ur2[i2] >= 0
                if only_stereo and not st2:
                    continue
                d = int(np.unpackbits(np.bitwise_xor(d1[i1], d2[i2])).sum())
                if d > TH_LOW or d > best_d:
                    continue
                if not st1 and not st2:
                    ex, ey = f32(f32(ep[0]) - k2["x"][i2]), f32(f32(ep[1]) - k2["y"][i2])
                    if sq2(ex, ey, fma) < f32(100 * scale2[k2["octave"][i2]]):
                        continue
                ok = bool(coarse)
                if not ok:
                    la = lin2(k1["x"][i1], F[0], k1["y"][i1], F[3], F[6], fma)
                    lb = lin2(k1["x"][i1], F[1], k1["y"][i1], F[4], F[7], fma)
                    lc = lin2(k1["x"][i1], F[2], k1["y"][i1], F[5], F[8], fma)
                    num = lin2(la, k2["x"][i2], lb, k2["y"][i2], lc, fma)
                    den = sq2(la, lb, fma)
                    if den != 0:
                        ok = float(f32(f32(num * num) / den)) < 3.84 * float(sigma2_2[k2["octave"][i2]])
                if ok:
                    best, best_d = i2, d
            if best >= 0:
                m12[i1] = best
                if check_ori:
                    hist[rot_bin(k1["angle"][i1], k2["angle"][best])].append(i1)
    if check_ori:
        keep = three_maxima([len(h) for h in hist])
        for b in range(HISTO):
            if b not in keep:
                for i1 in hist[b]:
                    m12[i1] = -1
    return m12
