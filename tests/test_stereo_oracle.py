"""Frame::ComputeStereoMatches: the C++ oracle against the independent numpy
restatement (tests/stereo_ref.py) on synthetic rectified pairs (C3 shape:
752x480, 1200 features, lapping {0,0}), bit-exact mvuRight / mvDepth."""
import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import synth
from tests.stereo_ref import stereo_matches

FX, BASE = 435.2, 0.11
MBF = float(np.float32(BASE) * np.float32(FX))


def pyramid(ex):
    return [ex.level(l) for l in range(8)]


@pytest.mark.parametrize("seed,w,h,nf", [(3000, 752, 480, 1200), (3001, 752, 480, 1200), (3100, 320, 240, 500)])
def test_oracle_stereo_vs_numpy(seed, w, h, nf):
    left, right = synth.stereo_pair(w, h, seed)
    el, er = O.OracleExtractor(nf, 1.2, 8, 20, 7), O.OracleExtractor(nf, 1.2, 8, 20, 7)
    kl, dl, _ = el(left, (0, 0))
    kr, dr, _ = er(right, (0, 0))
    t = el.tables()
    ur, dep = O.compute_stereo_matches(el, er, kl, dl, kr, dr, BASE, MBF)
    rur, rdep = stereo_matches(pyramid(el), pyramid(er), kl, dl, kr, dr, t["scale"], t["inv_scale"], BASE,
                               MBF)
    assert (ur >= 0).sum() > len(kl) // 4          # the synthetic disparity is found
    np.testing.assert_array_equal(ur.view(np.uint32), rur.view(np.uint32))
    np.testing.assert_array_equal(dep.view(np.uint32), rdep.view(np.uint32))


def test_oracle_stereo_no_right_keypoints():
    left, right = synth.stereo_pair(320, 240, 3200)
    el, er = O.OracleExtractor(300, 1.2, 8, 20, 7), O.OracleExtractor(300, 1.2, 8, 20, 7)
    kl, dl, _ = el(left, (0, 0))
    er(right, (0, 0))
    ur, dep = O.compute_stereo_matches(el, er, kl, dl, kl[:0], dl[:0], BASE, MBF)
    assert (ur == -1).all() and (dep == -1).all()


def knn2_numpy(q, t):
    """BFMatcher knnMatch(k=2) restated with a stable lexicographic sort."""
    if len(t) == 0:
        return np.full((len(q), 2), -1, np.int32), np.full((len(q), 2), -1, np.int32)
    d = np.unpackbits(np.bitwise_xor(q[:, None, :], t[None, :, :]), axis=-1).sum(-1)
    order = np.argsort(d, axis=1, kind="stable")[:, :2]
    idx = np.full((len(q), 2), -1, np.int32)
    dist = np.full((len(q), 2), -1, np.int32)
    k = min(2, len(t))
    idx[:, :k] = order[:, :k]
    dist[:, :k] = np.take_along_axis(d, order[:, :k], 1)
    return idx, dist


@pytest.mark.parametrize("nq,nt,seed", [(300, 280, 1), (50, 1, 2), (40, 0, 3), (200, 200, 4)])
def test_oracle_knn2_vs_numpy(nq, nt, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (max(nt, 1), 32), dtype=np.uint8)
    t = base[:nt].copy()
    if nt > 3:
        t[1] = t[0]                                    # duplicate rows: equal distances, index order
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    if nt:
        q[: nq // 2] = t[rng.integers(0, nt, nq // 2)] ^ (rng.random((nq // 2, 32)) < 0.03).astype(np.uint8)
    i, d = O.knn_match2(q, t)
    ri, rd = knn2_numpy(q, t)
    np.testing.assert_array_equal(i, ri)
    np.testing.assert_array_equal(d, rd)
