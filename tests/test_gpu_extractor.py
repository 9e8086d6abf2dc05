"""GPU parity of the HIP extractor against the CPU oracle: keypoints (all 28
bytes) and descriptors bit-exact, monoIndex equal, on the configs of
BASELINE.json and on edge cases; plus full-size properties."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, orb, synth

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


_cache = {}


def pair(nf=1000, sf=1.2, nl=8, ini=20, mn=7, blur=0, fma=1):
    key = (nf, sf, nl, ini, mn, blur, fma)
    if key not in _cache:
        _cache[key] = (orb.ORBextractor(nf, sf, nl, ini, mn, blur_variant=blur, fma_sampling=fma),
                       O.OracleExtractor(nf, sf, nl, ini, mn, blur, fma))
    return _cache[key]


def assert_same(img, lap, **kw):
    ex, ref = pair(**kw)
    k, d, m = ex(img, None, lap)
    rk, rd, rm = ref(img, lap)
    assert (len(k), m) == (len(rk), rm)
    assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)), "keypoints differ"
    assert np.array_equal(d, rd), "descriptors differ"
    return k, d, m


@pytest.mark.parametrize("i", range(4))
def test_c2_sequence_frames(gpu_lib, i):
    seq = synth.sequence(752, 480, 4, config=2, start=100)
    k, _, m = assert_same(seq[i], (0, 1000))
    assert len(k) >= 1000 and m == 0


@pytest.mark.parametrize("lap", [(0, 0), (200, 500), (0, 751), (-5, 10), (700, 800)])
def test_lapping_area(gpu_lib, lap):
    assert_same(synth.image(752, 480, 31), lap)


def test_c3_stereo_pair(gpu_lib):
    l, r = synth.stereo_pair(752, 480, 3000)
    assert_same(l, (0, 0), nf=1200)
    assert_same(r, (0, 0), nf=1200)


def test_c4_fisheye_512(gpu_lib):
    assert_same(synth.image(512, 512, 4000), (0, 511), nf=1500)


def test_c5_1080p(gpu_lib):
    assert_same(synth.image(1920, 1080, 5000), (0, 1000), nf=5000)


@pytest.mark.parametrize("kw", [dict(nf=500), dict(nf=2000, sf=1.3, nl=6, ini=15, mn=5), dict(nl=4),
                                dict(nl=1), dict(blur=1), dict(fma=0), dict(ini=40, mn=30)])
def test_parameter_variants(gpu_lib, kw):
    assert_same(synth.image(640, 480, 77), (0, 1000), **kw)


def test_flat_and_saturated_images(gpu_lib):
    k, _, m = assert_same(np.full((480, 752), 128, np.uint8), (0, 1000))
    assert len(k) == 0 and m == 0
    chk = ((np.indices((480, 752)).sum(0) // 7) % 2 * 255).astype(np.uint8)
    assert_same(chk, (0, 1000))
    noise = np.random.default_rng(0).integers(0, 256, (480, 752), dtype=np.uint8)
    assert_same(noise, (0, 1000))


def test_small_image(gpu_lib):
    assert_same(synth.image(160, 120, 5), (0, 1000), nl=3)


def test_empty_image_returns_minus_one(gpu_lib):
    ex, _ = pair()
    k, d, m = ex(np.zeros((0, 0), np.uint8), None, (0, 1000))
    assert m == -1 and len(k) == 0


def test_pyramid_and_stages(gpu_lib):
    ex, ref = pair()
    img = synth.image(752, 480, 12)
    ex(img, None, (0, 1000))
    ref(img, (0, 1000))
    for l, lev in enumerate(ex.mvImagePyramid):
        np.testing.assert_array_equal(lev, ref.level(l))
    for stage in (0, 1):
        for a, b in zip(ex.debug_stage(stage), ref.stage(stage)):
            np.testing.assert_array_equal(np.stack([a["x"], a["y"], a["response"]]),
                                          np.stack([b["x"], b["y"], b["response"]]))


def test_tables_match_oracle(gpu_lib):
    ex, ref = pair()
    t = ref.tables()
    np.testing.assert_array_equal(ex.GetScaleFactors(), t["scale"])
    np.testing.assert_array_equal(ex.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
    np.testing.assert_array_equal(ex.FeaturesPerLevel(), t["features"])
    np.testing.assert_array_equal(ex.UMax(), t["umax"])


@pytest.mark.parametrize("case", json.loads((G / "manifest.json").read_text())["cases"],
                         ids=lambda c: f"{c['name']}-{c['seed']}")
def test_golden_fixtures(gpu_lib, case):
    img = synth.image(case["w"], case["h"], case["seed"])
    ex, _ = pair(nf=case["nfeatures"])
    k, d, m = ex(img, None, tuple(case["lapping"]))
    assert (len(k), m) == (case["n"], case["mono"])
    assert sha(k) == case["kps_sha"] and sha(d) == case["desc_sha"]


def test_batch_device_equals_single(gpu_lib):
    import torch
    ex, _ = pair()
    seq = synth.sequence(752, 480, 12, config=9)
    kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
    torch.cuda.synchronize()
    for i in range(len(seq)):
        k, d, m = ex(seq[i], None, (0, 1000))
        ni = int(n[i])
        assert ni == len(k) and int(mono[i]) == m
        kb = orb.keypoints_from_device(kps[i, :ni])
        assert np.array_equal(kb.view(np.uint8), k.view(np.uint8))
        assert np.array_equal(desc[i, :ni].cpu().numpy(), d)


def test_full_size_batch_properties(gpu_lib):
    """64 frames at the bench size: deterministic, within capacity, every
    keypoint inside the detection borders of its level, per-level counts
    bounded by the quadtree (N + 2, or 4 initial nodes)."""
    import torch
    ex, _ = pair()
    seq = torch.from_numpy(synth.sequence(752, 480, 64, config=10)).cuda()
    a = [t.clone() for t in ex.extract_batch_device(seq, (0, 1000))[:4]]
    b = ex.extract_batch_device(seq, (0, 1000))
    torch.cuda.synchronize()
    for x, y in zip(a, b[:4]):
        assert torch.equal(x, y)
    cap = b[4]
    n = a[2].cpu().numpy()
    assert (n <= cap).all() and (n > 900).all()
    feats = ex.FeaturesPerLevel()
    scales = ex.GetScaleFactors()
    for i in range(0, 64, 9):
        k = orb.keypoints_from_device(a[0][i, :n[i]])
        for l in range(8):
            kl = k[k["octave"] == l]
            assert len(kl) <= max(feats[l] + 2, 8)
            lw = np.rint(np.float32(752) / scales[l])
            x = kl["x"] / scales[l]
            assert (x >= 18.5).all() and (x <= lw - 19.5).all()
        assert (k["class_id"] == -1).all()


def test_extract_batch_host_images(gpu_lib):
    """orbx_extract_batch: a stereo pair plus two more frames, per-frame lapping
    areas (grouped into runs), one of them repeated; every frame identical to
    the oracle on the same image."""
    l, r = synth.stereo_pair(752, 480, 3000)
    seq = synth.sequence(752, 480, 2, config=2, start=300)
    imgs = [l, r, seq[0], seq[1]]
    laps = [(0, 0), (0, 0), (200, 500), (0, 1000)]
    ex, ref = pair()
    out = ex.extract_batch(imgs, laps)
    for im, lap, (k, d, m) in zip(imgs, laps, out):
        rk, rd, rm = ref(im, lap)
        assert (len(k), m) == (len(rk), rm)
        assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)), "keypoints differ"
        assert np.array_equal(d, rd), "descriptors differ"
    # default lapping ({0, 1000}) and a single frame
    (k, d, m), = ex.extract_batch([seq[1]])
    rk, rd, rm = ref(seq[1], (0, 1000))
    assert (len(k), m) == (len(rk), rm) and np.array_equal(d, rd)


@pytest.mark.parametrize("host_pyr", [False, True])
def test_mvimagepyramid_host_and_device_copies(gpu_lib, host_pyr):
    """mvImagePyramid (include/ORBextractor.h:83) after orbx_extract, read
    through orbx_get_level either from the device or -- with
    orbx_set_host_pyramid -- from the copy the extraction graph downloads;
    both equal the oracle's ComputePyramid levels, frame after frame, and a
    later batch call or a toggle never serves a stale copy."""
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    ex.set_host_pyramid(host_pyr)
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    for f in range(3):
        img = synth.image(752, 480, synth.frame_seed(9, f))
        ex(img, None, (0, 1000))
        ref(img, (0, 1000))
        for lev, a in enumerate(ex.mvImagePyramid):
            np.testing.assert_array_equal(a, ref.level(lev), err_msg=f"frame {f} level {lev}")
    ex.set_host_pyramid(not host_pyr)
    img = synth.image(752, 480, synth.frame_seed(9, 7))
    ex(img, None, (0, 1000))
    ref(img, (0, 1000))
    for lev, a in enumerate(ex.mvImagePyramid):
        np.testing.assert_array_equal(a, ref.level(lev), err_msg=f"toggled, level {lev}")


@pytest.mark.parametrize("capopt", [1, 41, 400])
def test_fast_dense_cells(gpu_lib, capopt):
    """k_fast_cells' dense form (a cell whose pre-test candidates overflow the
    LDS list is scored at every window pixel and NMS-walked in row-major order,
    ORBextractor.cc:826-846 with cv::FAST's own definition): the candidate list
    capped at capopt - 1 entries through the ORB_OPT_FAST_CAND_CAP hook (1:
    every cell holding a candidate goes dense; 41 / 400: a mix), on textured,
    checkerboard and uniform-noise frames, in both the ROI pre-test and the
    fused-bitmap forms: keypoints and descriptors equal the oracle's."""
    import torch
    from orb_slam3_vio_fixes_amd import capi
    chk = ((np.indices((480, 752)).sum(0) // 5) % 2 * 255).astype(np.uint8)
    noise = np.random.default_rng(7).integers(0, 256, (480, 752), dtype=np.uint8)
    imgs = [synth.image(752, 480, 4321), chk, noise]
    with capi.debug_option(capi.ORB_OPT_FAST_CAND_CAP, capopt):
        for img in imgs:
            assert_same(img, (0, 1000))
        with capi.debug_option(capi.ORB_OPT_PYR_PRETEST, 1):
            ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
            ex.set_pyramid_mode(2)
            seq = np.stack(imgs)
            kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
            torch.cuda.synchronize()
        assert ex.plan_info(752, 480)["pretest"] == 1
        ref = pair()[1]
        for f in range(len(seq)):
            rk, rd, rm = ref(seq[f], (0, 1000))
            ni = int(n[f])
            assert (ni, int(mono[f])) == (len(rk), rm)
            kb = orb.keypoints_from_device(kps[f, :ni])
            assert np.array_equal(kb.view(np.uint8), rk.view(np.uint8)), f"frame {f}: keypoints differ"
            assert np.array_equal(desc[f, :ni].cpu().numpy(), rd), f"frame {f}: descriptors differ"
