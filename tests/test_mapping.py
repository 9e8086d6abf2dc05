"""Mapping-thread matchers: Fuse(pKF, vpMapPoints, th)
and SearchForTriangulation for pinhole keyframes.  CPU: the oracle against the
independent Python restatement (tests/mapping_ref.py); GPU: the HIP kernels
against the oracle.  Keyframes are consecutive frames of a synthetic panning
sequence (C2 shape), FeatureVectors from a synthetic k=10, L=6 vocabulary."""
import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, synth
from tests import mapping_ref as R

W, H = 752, 480


def F12_and_ep():
    K = np.array([[435.2, 0, 376.0], [0, 435.2, 240.0], [0, 0, 1]])
    a = 0.03
    Rm = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    t = np.array([0.1, 0.01, 0.02])
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Ki = np.linalg.inv(K)
    F = (Ki.T @ tx @ Rm @ Ki).astype(np.float32)
    return F, (np.float32(400.0), np.float32(240.0))


@pytest.fixture(scope="module")
def scene():
    frames = synth.sequence(W, H, 2, config=2, start=4000)
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    t = ex.tables()
    kfs = [ex(f, (0, 0))[:2] for f in frames]
    voc = abi.vocab_struct(synth.vocabulary(10, 6, seed=31))
    nids = [O.transform(voc, d, 4)[2] for _, d in kfs]
    return kfs, nids, t


def featvec_dict(nid):
    fv = {}
    for i, n in enumerate(nid.tolist()):
        fv.setdefault(n, []).append(i)
    return fv


def tri_inputs(scene, stereo, seed):
    (k1, d1), (k2, d2) = scene[0]
    rng = np.random.default_rng(seed)
    mp1 = (rng.random(len(k1)) < 0.25).astype(np.uint8)
    mp2 = (rng.random(len(k2)) < 0.25).astype(np.uint8)
    ur1 = np.where(rng.random(len(k1)) < 0.6, k1["x"] - rng.uniform(0, 40, len(k1)), -1).astype(np.float32) \
        if stereo else None
    ur2 = np.where(rng.random(len(k2)) < 0.6, k2["x"] - rng.uniform(0, 40, len(k2)), -1).astype(np.float32) \
        if stereo else None
    return k1, d1, k2, d2, mp1, mp2, ur1, ur2


@pytest.mark.parametrize("stereo,only_stereo,coarse,seed", [(False, False, False, 1), (True, False, False, 2),
                                                            (True, True, False, 3), (False, False, True, 4)])
def test_oracle_triangulation_vs_python(scene, stereo, only_stereo, coarse, seed):
    k1, d1, k2, d2, mp1, mp2, ur1, ur2 = tri_inputs(scene, stereo, seed)
    nid1, nid2 = scene[1]
    t = scene[2]
    F, ep = F12_and_ep()
    f1 = abi.frame_struct(k1, d1, W, H, u_right=ur1, scale_factors=t["scale"])
    f2 = abi.frame_struct(k2, d2, W, H, u_right=ur2, scale_factors=t["scale"])
    nm, m12 = O.search_for_triangulation(f1, abi.featvec_struct(nid1), mp1, f2, abi.featvec_struct(nid2), mp2, F, ep,
                                         t["sigma2"], only_stereo, coarse, True)
    ref = R.search_for_triangulation(k1, d1, ur1, mp1, featvec_dict(nid1), k2, d2, ur2, mp2, featvec_dict(nid2),
                                     t["scale"], t["sigma2"], F, ep, only_stereo, coarse, True)
    np.testing.assert_array_equal(m12, ref)
    assert nm == (ref >= 0).sum() and nm > (5 if only_stereo else 20)


def fuse_inputs(scene, stereo, seed):
    k, d = scene[0][1]
    rng = np.random.default_rng(seed)
    n = len(k)
    u = (k["x"] + rng.normal(0, 1.5, n)).astype(np.float32)
    v = (k["y"] + rng.normal(0, 1.5, n)).astype(np.float32)
    ur = (u - rng.uniform(5, 30, n)).astype(np.float32)
    level = np.minimum(k["octave"] + rng.integers(0, 2, n), 7).astype(np.int32)
    bits = np.unpackbits(d, axis=1)
    md = np.packbits(bits ^ (rng.random(bits.shape) < 0.05), axis=1)
    valid = (rng.random(n) < 0.9).astype(np.uint8)
    kur = np.where(rng.random(n) < 0.5, ur + rng.normal(0, 1, n), -1).astype(np.float32) if stereo else None
    return k, d, kur, u, v, ur, level, md, valid


@pytest.mark.parametrize("stereo,seed", [(False, 5), (True, 6)])
def test_oracle_fuse_vs_python(scene, stereo, seed):
    k, d, kur, u, v, ur, level, md, valid = fuse_inputs(scene, stereo, seed)
    t = scene[2]
    f = abi.frame_struct(k, d, W, H, u_right=kur, scale_factors=t["scale"])
    nf, bi, bd = O.fuse(f, t["inv_sigma2"], valid, u, v, ur, level, md, 3.0)
    grid = R.make_grid(k, 0.0, W, 0.0, H)
    ref = R.fuse(k, d, kur, t["scale"], t["inv_sigma2"], grid, valid, u, v, ur, level, md, 3.0)
    np.testing.assert_array_equal(bi, ref)
    assert nf == (ref >= 0).sum() and nf > 100


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,only_stereo,coarse,seed", [(False, False, False, 1), (True, False, False, 2),
                                                            (True, True, False, 3), (False, False, True, 4)])
def test_gpu_triangulation(gpu_lib, scene, stereo, only_stereo, coarse, seed):
    from orb_slam3_vio_fixes_amd import orb
    k1, d1, k2, d2, mp1, mp2, ur1, ur2 = tri_inputs(scene, stereo, seed)
    nid1, nid2 = scene[1]
    t = scene[2]
    F, ep = F12_and_ep()
    f1 = abi.frame_struct(k1, d1, W, H, u_right=ur1, scale_factors=t["scale"])
    f2 = abi.frame_struct(k2, d2, W, H, u_right=ur2, scale_factors=t["scale"])
    fv1, fv2 = abi.featvec_struct(nid1), abi.featvec_struct(nid2)
    rn, rm = O.search_for_triangulation(f1, fv1, mp1, f2, fv2, mp2, F, ep, t["sigma2"], only_stereo, coarse, True)
    gn, gm = orb.ORBmatcher(0.6, True).SearchForTriangulation(f1, fv1, mp1, f2, fv2, mp2, F, ep, t["sigma2"],
                                                             only_stereo, coarse)
    assert gn == rn
    np.testing.assert_array_equal(gm, rm)


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,seed", [(False, 5), (True, 6)])
def test_gpu_fuse(gpu_lib, scene, stereo, seed):
    from orb_slam3_vio_fixes_amd import orb
    k, d, kur, u, v, ur, level, md, valid = fuse_inputs(scene, stereo, seed)
    t = scene[2]
    f = abi.frame_struct(k, d, W, H, u_right=kur, scale_factors=t["scale"])
    rn, rb, rd = O.fuse(f, t["inv_sigma2"], valid, u, v, ur, level, md, 3.0)
    gn, gb, gd = orb.ORBmatcher.Fuse(f, t["inv_sigma2"], valid, u, v, ur, level, md, 3.0)
    assert gn == rn
    np.testing.assert_array_equal(gb, rb)
    np.testing.assert_array_equal(gd, rd)


def distinctive_sets(seed):
    rng = np.random.default_rng(seed)
    sizes = [1, 2, 3, 4, 5, 8, 17, 40, 64, 65, 130, 300] + list(rng.integers(1, 60, 60))
    base = rng.integers(0, 256, (len(sizes), 32), dtype=np.uint8)
    rows = []
    for p, n in enumerate(sizes):
        bits = np.unpackbits(np.repeat(base[p][None], n, 0), axis=1)
        flips = rng.random(bits.shape) < rng.uniform(0.02, 0.3)
        d = np.packbits(bits ^ flips, axis=1)
        if n > 3:
            d[1] = d[0]                                  # ties between rows
        rows.append(d)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    return off, np.concatenate(rows)


def distinctive_python(off, desc):
    out = []
    for p in range(len(off) - 1):
        d = desc[off[p]:off[p + 1]]
        n = len(d)
        m = np.unpackbits(np.bitwise_xor(d[:, None, :], d[None, :, :]), axis=-1).sum(-1)
        med = np.sort(m, axis=1)[:, int(0.5 * (n - 1))]
        out.append(int(np.argmin(med)))                  # first least median
    return np.array(out, np.int32)


def test_oracle_distinctive_vs_python():
    off, desc = distinctive_sets(7)
    np.testing.assert_array_equal(O.compute_distinctive_descriptors(off, desc), distinctive_python(off, desc))


@pytest.mark.gpu
def test_gpu_distinctive(gpu_lib):
    from orb_slam3_vio_fixes_amd import orb
    off, desc = distinctive_sets(8)
    np.testing.assert_array_equal(orb.compute_distinctive_descriptors(off, desc),
                                  O.compute_distinctive_descriptors(off, desc))
    edge = np.array([0, 0, 3], np.int32)                 # a point without descriptors, then one with three
    got = orb.compute_distinctive_descriptors(edge, desc[:3])
    assert got[0] == -1
    np.testing.assert_array_equal(got, O.compute_distinctive_descriptors(edge, desc[:3]))


# ---- SearchForTriangulation with the caller's geometry (KannalaBrandt8 / two-camera keyframes) ----

def _tri_predicates(k1, k2):
    """Pure per-candidate checks standing in for epipolarConstrain: accept all,
    an arbitrary hash (ties between equal distances matter), and a row-band
    constraint (a geometric stand-in for the panning pair)."""
    return {
        "all": lambda i1, i2: True,
        "hash": lambda i1, i2: (i1 * 2654435761 + i2 * 40503) % 7 != 0,
        "band": lambda i1, i2: abs(float(k1[i1]["y"]) - float(k2[i2]["y"])) < 6.0 + 2.0 * int(k2[i2]["octave"]),
    }


def ref_tri_checked(k1, d1, ur1, mp1, fv1, k2, d2, ur2, mp2, fv2, only_stereo, check):
    """The reference loop (ORBmatcher.cc:962-1144), the callback in place of the
    epipole test and epipolarConstrain; independent of the C++ oracle."""
    from tests import matcher_ref as M
    m12 = np.full(len(k1), -1, np.int32)
    hist = [[] for _ in range(M.HISTO)]
    nm = 0
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if mp1[i1]:
                continue
            st1 = ur1 is not None and ur1[i1] >= 0
            if only_stereo and not st1:
                continue
            best, bi = M.TH_LOW, -1
            for i2 in fv2[node]:
                if mp2[i2]:
                    continue
                st2 = ur2 is not None and ur2[i2] >= 0
                if only_stereo and not st2:
                    continue
                dist = M.hamming(d1[i1], d2[i2])
                if dist > M.TH_LOW or dist > best:
                    continue
                if check(i1, i2):
                    best, bi = dist, i2
            if bi >= 0:
                m12[i1] = bi
                nm += 1
                hist[M.rot_bin(k1[i1]["angle"], k2[bi]["angle"])].append(i1)
    keep = M.three_maxima([len(h) for h in hist])
    for b in range(M.HISTO):
        if b not in keep:
            for i1 in hist[b]:
                m12[i1] = -1
                nm -= 1
    return nm, m12


@pytest.mark.parametrize("stereo,only_stereo,pred,seed", [(False, False, "hash", 11), (True, False, "band", 12),
                                                           (True, True, "hash", 13), (False, False, "band", 14)])
def test_oracle_triangulation_checked_vs_python(scene, stereo, only_stereo, pred, seed):
    k1, d1, k2, d2, mp1, mp2, ur1, ur2 = tri_inputs(scene, stereo, seed)
    nid1, nid2 = scene[1]
    t = scene[2]
    f1 = abi.frame_struct(k1, d1, W, H, u_right=ur1, scale_factors=t["scale"])
    f2 = abi.frame_struct(k2, d2, W, H, u_right=ur2, scale_factors=t["scale"])
    check = _tri_predicates(k1, k2)[pred]
    nm, m12 = O.search_for_triangulation_checked(f1, abi.featvec_struct(nid1), mp1, f2, abi.featvec_struct(nid2),
                                                 mp2, check, only_stereo)
    rn, rm = ref_tri_checked(k1, d1, ur1, mp1, featvec_dict(nid1), k2, d2, ur2, mp2, featvec_dict(nid2),
                             only_stereo, check)
    assert nm == rn and nm > 0
    np.testing.assert_array_equal(m12, rm)


@pytest.mark.parametrize("stereo", [False, True])
def test_oracle_triangulation_checked_accept_all_is_coarse(scene, stereo):
    """With a check that accepts everything and the epipole out of reach, the
    checked form is the pinhole form with bCoarse."""
    k1, d1, k2, d2, mp1, mp2, ur1, ur2 = tri_inputs(scene, stereo, 15)
    nid1, nid2 = scene[1]
    t = scene[2]
    F, _ = F12_and_ep()
    f1 = abi.frame_struct(k1, d1, W, H, u_right=ur1, scale_factors=t["scale"])
    f2 = abi.frame_struct(k2, d2, W, H, u_right=ur2, scale_factors=t["scale"])
    fv1, fv2 = abi.featvec_struct(nid1), abi.featvec_struct(nid2)
    a = O.search_for_triangulation_checked(f1, fv1, mp1, f2, fv2, mp2, lambda i1, i2: True)
    b = O.search_for_triangulation(f1, fv1, mp1, f2, fv2, mp2, F, (-1e6, -1e6), t["sigma2"], False, True, True)
    assert a[0] == b[0] and a[0] > 0
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,only_stereo,pred,seed", [(False, False, "all", 21), (False, False, "hash", 22),
                                                           (True, False, "band", 23), (True, True, "hash", 24)])
def test_gpu_triangulation_checked(gpu_lib, scene, stereo, only_stereo, pred, seed):
    from orb_slam3_vio_fixes_amd import orb
    k1, d1, k2, d2, mp1, mp2, ur1, ur2 = tri_inputs(scene, stereo, seed)
    nid1, nid2 = scene[1]
    t = scene[2]
    f1 = abi.frame_struct(k1, d1, W, H, u_right=ur1, scale_factors=t["scale"])
    f2 = abi.frame_struct(k2, d2, W, H, u_right=ur2, scale_factors=t["scale"])
    fv1, fv2 = abi.featvec_struct(nid1), abi.featvec_struct(nid2)
    check = _tri_predicates(k1, k2)[pred]
    rn, rm = O.search_for_triangulation_checked(f1, fv1, mp1, f2, fv2, mp2, check, only_stereo)
    gn, gm = orb.ORBmatcher(0.6, True).SearchForTriangulationChecked(f1, fv1, mp1, f2, fv2, mp2, check, only_stereo)
    assert gn == rn and gn > 0
    np.testing.assert_array_equal(gm, rm)
