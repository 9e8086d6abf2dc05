"""Independent pure-Python restatements of the matchers' fisheye-stereo
branches (Frame::Nleft != -1), used to pin the C++ oracle:
SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:223-425, :296-323,
:357-386), SearchByProjection(Frame&, vector<MapPoint*>) (:43-213) and
SearchByProjection(Frame&, const Frame&) (:1676-1887).  The frame is the
combined keypoint array [mvKeys (nleft); mvKeysRight] with mGrid over the
left keypoints and mGridRight over the right ones by local index
(Frame.cc:385-416)."""
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


def _radius_by_viewing_cos(c):
    return f32(2.5) if c > 0.998 else f32(4.0)


def search_by_bow_fisheye(kk, kd, kfv, kvalid, fk, fd, ffv, nleft, ratio, check_ori):
    match = [-1] * len(fk)
    hist = [[] for _ in range(HISTO)]
    nm = 0
    for node in sorted(set(kfv) & set(ffv)):
        for ikf in kfv[node]:
            if not kvalid[ikf]:
                continue
            b1 = b2 = b1r = b2r = 256
            bi = bir = -1
            for jf in ffv[node]:
                if match[jf] >= 0:
                    continue
                dist = M.hamming(kd[ikf], fd[jf])
                if jf < nleft and dist < b1:
                    b2, b1, bi = b1, dist, jf
                elif jf < nleft and dist < b2:
                    b2 = dist
                if jf >= nleft and dist < b1r:
                    b2r, b1r, bir = b1r, dist, jf
                elif jf >= nleft and dist < b2r:
                    b2r = dist
            if b1 <= TH_LOW:
                if f32(b1) < f32(f32(ratio) * f32(b2)):
                    match[bi] = ikf
                    if check_ori:
                        hist[M.rot_bin(kk[ikf]["angle"], fk[bi]["angle"])].append(bi)
                    nm += 1
                if b1r <= TH_LOW:
                    match[bir] = ikf
                    if check_ori:
                        hist[M.rot_bin(kk[ikf]["angle"], fk[bir]["angle"])].append(bir)
                    nm += 1
    if check_ori:
        nm = _rot_filter(hist, match, nm)
    return nm, np.array(match, np.int32)


def _best2(k, d, cand, off, qd, blocked_slot):
    best = best2 = 256
    bl = bl2 = bi = -1
    for idx in cand:
        slot = idx + off
        if blocked_slot(slot):
            continue
        dist = M.hamming(qd, d[slot])
        if dist < best:
            best2, bl2 = best, bl
            best, bl, bi = dist, int(k[slot]["octave"]), idx
        elif dist < best2:
            bl2, best2 = int(k[slot]["octave"]), dist
    return best, bl, best2, bl2, bi


def search_by_projection_mps_fisheye(k, d, w, h, scale, nleft, l2r, r2l, q, qr, th, far, th_far, ratio, owner,
                                     blocked):
    """q: dict in_view, x, y, level, view_cos, depth, has_obs, desc (left); qr: in_view, x, y, level, view_cos."""
    kl, kr = k[:nleft], k[nleft:]
    gl, gr = M.grid(kl, w, h), M.grid(kr, w, h)
    owner = [int(o) for o in owner]

    def blk(slot):
        o = owner[slot]
        if o == -1:
            return False
        return bool(blocked[slot]) if o <= -2 else bool(q["has_obs"][o])

    nm = 0
    for i in range(len(q["in_view"])):
        if not q["in_view"][i] and not qr["in_view"][i]:
            continue
        if far and q["depth"][i] > th_far:
            continue
        if q["in_view"][i]:
            lvl = int(q["level"][i])
            r = _radius_by_viewing_cos(q["view_cos"][i])
            if th != 1.0:
                r = f32(r * f32(th))
            cand = M.area(kl, gl, q["x"][i], q["y"][i], f32(r * f32(scale[lvl])), lvl - 1, lvl)
            if cand:
                best, bl, best2, bl2, bi = _best2(k, d, cand, 0, q["desc"][i], blk)
                if best <= TH_HIGH:
                    if bl == bl2 and f32(best) > f32(f32(ratio) * f32(best2)):
                        continue
                    owner[bi] = i
                    if l2r[bi] != -1:
                        owner[l2r[bi] + nleft] = i
                        nm += 1
                    nm += 1
        if qr["in_view"][i]:
            lvl = int(qr["level"][i])
            if lvl != -1:
                r = _radius_by_viewing_cos(qr["view_cos"][i])
                cand = M.area(kr, gr, qr["x"][i], qr["y"][i], f32(r * f32(scale[lvl])), lvl - 1, lvl)
                if not cand:
                    continue
                best, bl, best2, bl2, bi = _best2(k, d, cand, nleft, q["desc"][i], blk)
                if best <= TH_HIGH:
                    if bl == bl2 and f32(best) > f32(f32(ratio) * f32(best2)):
                        continue
                    if r2l[bi] != -1:
                        owner[r2l[bi]] = i
                        nm += 1
                    owner[bi + nleft] = i
                    nm += 1
    return nm, np.array(owner, np.int32)


def search_by_projection_last_fisheye(k, d, w, h, scale, nleft, valid, u, v, ur, vr, octave, angle, has_obs, desc,
                                      th, mode, check_ori, owner, blocked):
    kl, kr = k[:nleft], k[nleft:]
    gl, gr = M.grid(kl, w, h), M.grid(kr, w, h)
    owner = [int(o) for o in owner]
    hist = [[] for _ in range(HISTO)]

    def blk(slot):
        o = owner[slot]
        if o == -1:
            return False
        return bool(blocked[slot]) if o <= -2 else bool(has_obs[o])

    def area(kk, g, x, y, r, oct):
        if mode == 1:
            return M.area(kk, g, x, y, r, oct, -1)
        if mode == 2:
            return M.area(kk, g, x, y, r, 0, oct)
        return M.area(kk, g, x, y, r, oct - 1, oct + 1)

    nm = 0
    for i in range(len(valid)):
        if not valid[i]:
            continue
        oct = int(octave[i])
        radius = f32(f32(th) * f32(scale[oct]))
        cand = area(kl, gl, u[i], v[i], radius, oct)
        if not cand:
            continue
        best, bi = 256, -1
        for i2 in cand:
            if blk(i2):
                continue
            dist = M.hamming(desc[i], d[i2])
            if dist < best:
                best, bi = dist, i2
        if best <= TH_HIGH:
            owner[bi] = i
            nm += 1
            if check_ori:
                hist[M.rot_bin(angle[i], k[bi]["angle"])].append(bi)
        best, bi = 256, -1
        for i2 in area(kr, gr, ur[i], vr[i], radius, oct):
            if blk(i2 + nleft):
                continue
            dist = M.hamming(desc[i], d[i2 + nleft])
            if dist < best:
                best, bi = dist, i2
        if best <= TH_HIGH:
            owner[bi + nleft] = i
            nm += 1
            if check_ori:
                hist[M.rot_bin(angle[i], k[bi + nleft]["angle"])].append(bi + nleft)
    if check_ori:
        nm = _rot_filter(hist, owner, nm)
    return nm, np.array(owner, np.int32)
