"""Independent pure-Python restatements of the relocalisation / loop-closing
matchers (small inputs only), used to pin the C++ oracle:
SearchByBoW(KeyFrame*, KeyFrame*) (src/ORBmatcher.cc:765-905),
SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (:1889-2010),
SearchByProjection(KeyFrame*, Sim3, vpPoints, vpMatched, th, ratioHamming)
(:427-532, and the vpPointsKFs twin :534-646), SearchBySim3 (:1457-1674),
Fuse(KeyFrame*, Sim3, vpPoints, th, vpReplacePoint) (:1340-1455).
Grid and candidate order from tests/matcher_ref.py (Frame.cc:657-735,
KeyFrame.cc:704-748); float32 arithmetic where the reference has float."""
import numpy as np

import matcher_ref as M

TH_HIGH, TH_LOW, HISTO = M.TH_HIGH, M.TH_LOW, M.HISTO
f32 = np.float32


def _rot_filter(hist, slots, nm):
    keep = M.three_maxima([len(x) for x in hist])
    for b in range(HISTO):
        if b in keep:
            continue
        for j in hist[b]:
            slots[j] = -1
            nm -= 1
    return nm


def search_by_bow_kf(k1, d1, fv1, valid1, k2, d2, fv2, valid2, ratio, check_ori):
    """fv1/fv2: dict node -> feature indices.  Returns (nmatches, matches12)."""
    m12 = [-1] * len(k1)
    matched2 = [False] * len(k2)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if not valid1[i1]:
                continue
            best = best2 = 256
            bi = -1
            for i2 in fv2[node]:
                if matched2[i2] or not valid2[i2]:
                    continue
                dist = M.hamming(d1[i1], d2[i2])
                if dist < best:
                    best2, best, bi = best, dist, i2
                elif dist < best2:
                    best2 = dist
            if best < TH_LOW and f32(best) < f32(f32(ratio) * f32(best2)):
                m12[i1] = bi
                matched2[bi] = True
                if check_ori:
                    hist[M.rot_bin(k1[i1]["angle"], k2[bi]["angle"])].append(i1)
                nm += 1
    if check_ori:
        nm = _rot_filter(hist, m12, nm)
    return nm, np.array(m12, np.int32)


def search_by_projection_kf(fk, fd, w, h, scale, valid, u, v, level, kf_angle, desc, th, orb_dist, check_ori,
                            owner):
    g = M.grid(fk, w, h)
    owner = [int(o) for o in owner]
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for i in range(len(valid)):
        if not valid[i]:
            continue
        pl = int(level[i])
        r = f32(f32(th) * f32(scale[pl]))
        cand = M.area(fk, g, u[i], v[i], r, pl - 1, pl + 1)
        best, bi = 256, -1
        for i2 in cand:
            if owner[i2] != -1:
                continue
            dist = M.hamming(desc[i], fd[i2])
            if dist < best:
                best, bi = dist, i2
        if bi >= 0 and best <= orb_dist:
            owner[bi] = i
            nm += 1
            if check_ori:
                hist[M.rot_bin(kf_angle[i], fk[bi]["angle"])].append(bi)
    if check_ori:
        nm = _rot_filter(hist, owner, nm)
    return nm, np.array(owner, np.int32)


def _best_in_area(kk, kd, g, scale, x, y, pl, d, th, skip=None):
    r = f32(f32(th) * f32(scale[pl]))
    best, bi = 2 ** 31 - 1, -1
    for idx in M.area(kk, g, x, y, r):
        if skip is not None and skip[idx] != -1:
            continue
        kl = int(kk[idx]["octave"])
        if kl < pl - 1 or kl > pl:
            continue
        dist = M.hamming(d, kd[idx])
        if dist < best:
            best, bi = dist, idx
    return best, bi


def search_by_projection_sim3(kk, kd, w, h, scale, valid, u, v, level, desc, th, ratio_hamming, matched):
    g = M.grid(kk, w, h)
    matched = [int(m) for m in matched]
    nm = 0
    for i in range(len(valid)):
        if not valid[i]:
            continue
        best, bi = _best_in_area(kk, kd, g, scale, u[i], v[i], int(level[i]), desc[i], th, skip=matched)
        if bi >= 0 and f32(best) <= f32(f32(TH_LOW) * f32(ratio_hamming)):
            matched[bi] = i
            nm += 1
    return nm, np.array(matched, np.int32)


def search_by_sim3(k1, d1, k2, d2, w, h, scale1, scale2, q1, q2, th):
    g1, g2 = M.grid(k1, w, h), M.grid(k2, w, h)
    vn1, vn2 = [-1] * len(k1), [-1] * len(k2)
    for i1 in range(len(k1)):
        va, u, v, lv, d = (x[i1] for x in q1)
        if va:
            best, bi = _best_in_area(k2, d2, g2, scale2, u, v, int(lv), d, th)
            if best <= TH_HIGH:
                vn1[i1] = bi
    for i2 in range(len(k2)):
        va, u, v, lv, d = (x[i2] for x in q2)
        if va:
            best, bi = _best_in_area(k1, d1, g1, scale1, u, v, int(lv), d, th)
            if best <= TH_HIGH:
                vn2[i2] = bi
    m12 = np.full(len(k1), -1, np.int32)
    for i1, i2 in enumerate(vn1):
        if i2 >= 0 and vn2[i2] == i1:
            m12[i1] = i2
    return int((m12 >= 0).sum()), m12


def fuse_sim3(kk, kd, w, h, scale, valid, u, v, level, desc, th):
    g = M.grid(kk, w, h)
    bi = np.full(len(valid), -1, np.int32)
    for i in range(len(valid)):
        if valid[i]:
            best, b = _best_in_area(kk, kd, g, scale, u[i], v[i], int(level[i]), desc[i], th)
            if best <= TH_LOW:
                bi[i] = b
    return int((bi >= 0).sum()), bi
