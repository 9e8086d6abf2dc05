"""Independent numpy restatement of Frame::ComputeStereoMatches
(reference src/Frame.cc:811-981), used to pin the C++ oracle
(tests/test_stereo_oracle.py).  Written from the reference semantics, not
from the oracle: the row table becomes a band test, the first-minimum scans
become explicit argmin-with-lowest-index, float32 arithmetic is kept where the
reference computes in float."""
from __future__ import annotations

import numpy as np

TH_HIGH, TH_LOW = 100, 50
f32 = np.float32


def _popcount_rows(x: np.ndarray) -> np.ndarray:
    return np.unpackbits(x, axis=-1).sum(axis=-1)


def _round_away(x: np.float32) -> np.float32:
    return f32(np.floor(np.float64(x) + 0.5)) if x >= 0 else f32(-np.floor(-np.float64(x) + 0.5))


def stereo_matches(pyr_l, pyr_r, kl, dl, kr, dr, scale, inv_scale, mb: float, mbf: float):
    nl = len(kl)
    ur = np.full(nl, -1.0, np.float32)
    dep = np.full(nl, -1.0, np.float32)
    th_orb = (TH_HIGH + TH_LOW) // 2
    mb, mbf = f32(mb), f32(mbf)
    max_d = f32(mbf / mb)
    min_d = f32(0.0)
    # right keypoints' row bands (:828-838)
    r_rad = (f32(2.0) * scale[kr["octave"]]).astype(np.float32)
    maxr = np.ceil((kr["y"] + r_rad).astype(np.float32)).astype(np.int64)
    minr = np.floor((kr["y"] - r_rad).astype(np.float32)).astype(np.int64)
    accepted = []
    for iL in range(nl):
        kp = kl[iL]
        lvl = int(kp["octave"])
        vL, uL = f32(kp["y"]), f32(kp["x"])
        row = int(vL)
        min_u, max_u = f32(uL - max_d), f32(uL - min_d)
        if max_u < 0:
            continue
        ok = (row >= minr) & (row <= maxr)
        ok &= (kr["octave"] >= lvl - 1) & (kr["octave"] <= lvl + 1)
        ok &= (kr["x"] >= min_u) & (kr["x"] <= max_u)
        idx = np.nonzero(ok)[0]
        if len(idx) == 0:
            continue
        dist = _popcount_rows(np.bitwise_xor(dr[idx], dl[iL][None, :]))
        keep = dist < TH_HIGH
        if not keep.any():
            continue
        best_dist = int(dist[keep].min())
        best_r = int(idx[keep][np.argmax(dist[keep] == best_dist)])     # first in index order
        if best_dist >= th_orb:
            continue
        sf = inv_scale[lvl]
        su_l = _round_away(f32(kp["x"] * sf))                  # std::round (half away from zero)
        sv_l = _round_away(f32(kp["y"] * sf))
        su_r0 = _round_away(f32(kr["x"][best_r] * sf))
        IL, IR = pyr_l[lvl], pyr_r[lvl]
        if su_r0 < 0 or su_r0 + 11 >= IR.shape[1]:
            continue
        y0, xl0 = int(sv_l) - 5, int(su_l) - 5
        patch_l = IL[y0:y0 + 11, xl0:xl0 + 11].astype(np.int64)
        dists = []
        for inc in range(-5, 6):
            xr0 = int(su_r0) + inc - 5
            dists.append(f32(np.abs(patch_l - IR[y0:y0 + 11, xr0:xr0 + 11].astype(np.int64)).sum()))
        dists = np.array(dists, np.float32)
        best_inc = int(np.argmin(dists)) - 5                     # first minimum
        best_sad = int(dists[best_inc + 5])
        if best_inc in (-5, 5):
            continue
        d1, d2, d3 = dists[best_inc + 4], dists[best_inc + 5], dists[best_inc + 6]
        with np.errstate(divide="ignore", invalid="ignore"):
            delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if delta < -1 or delta > 1:                             # NaN passes, then fails the disparity test
            continue
        best_ur = f32(scale[lvl] * f32(f32(f32(su_r0) + f32(best_inc)) + delta))
        disp = f32(uL - best_ur)
        if disp >= min_d and disp < max_d:
            if disp <= 0:
                disp = f32(0.01)
                best_ur = f32(np.float64(uL) - 0.01)
            dep[iL] = f32(mbf / disp)
            ur[iL] = best_ur
            accepted.append((best_sad, iL))
    if accepted:
        accepted.sort()
        median = f32(accepted[len(accepted) // 2][0])
        th = f32(f32(f32(1.5) * f32(1.4)) * median)
        for s, i in reversed(accepted):
            if f32(s) < th:
                break
            ur[i] = -1.0
            dep[i] = -1.0
    return ur, dep
