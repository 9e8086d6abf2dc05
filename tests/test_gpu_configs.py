"""BASELINE.json configurations run as whole workloads on the GPU against the
CPU oracle, plus the extractor-handle edge cases of the round-1 review:

* C3 exactly as stated: a 16-frame window of 752x480 stereo pairs (L+R),
  ORBextractor(1200) with lapping {0, 0}, extracted in ONE batch, then
  ComputeStereoMatches on the 16 pairs and SearchForInitialization over the
  15 consecutive left pairs — every keypoint, descriptor, mvuRight/mvDepth and
  matches12 entry compared with the oracle;
* the monocular initialization extractor at 752x480: Tracking builds it with
  5*nFeatures (src/Tracking.cc:601,1289) and uses it on the two frames that
  go into SearchForInitialization (:1586-1587, :2459-2492);
* plan errors that must repeat (no half-built plan), per-frame pyramids of a
  mixed-lapping batch, the threaded host gather of orbx_extract_batch with
  row steps wider than the image.
"""

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, capi, orb, synth

pytestmark = pytest.mark.gpu

FX, BASE = 435.2, 0.11
MBF = float(np.float32(BASE) * np.float32(FX))
INV_W = float(np.float32(64) / np.float32(752))
INV_H = float(np.float32(48) / np.float32(480))


def frame(k, d, nl=8):
    return abi.frame_struct(k, d, 752, 480, scale_factors=np.float32(1.2) ** np.arange(nl, dtype=np.float32))


def same_frame(k, d, m, rk, rd, rm):
    assert (len(k), m) == (len(rk), rm)
    assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)), "keypoints differ"
    assert np.array_equal(d, rd), "descriptors differ"


def test_c3_stereo_window(gpu_lib):
    import torch
    P = 16
    left, right = synth.stereo_sequence(752, 480, P, config=3, start=40)
    frames = torch.from_numpy(np.concatenate([left, right])).cuda()
    ex = orb.ORBextractor(1200, 1.2, 8, 20, 7)
    kps, desc, n, mono, cap = ex.extract_batch_device(frames, (0, 0))
    ur, dep, _ = orb.compute_stereo_matches_batch_device(ex, P, 0, P, kps, desc, n, cap, BASE, MBF)
    m = torch.empty((P - 1, cap), dtype=torch.int32, device="cuda")
    nm = torch.empty(P - 1, dtype=torch.int32, device="cuda")
    rc = capi.lib().orbm_search_for_initialization_batch_device(
        P, kps.data_ptr(), desc.data_ptr(), n.data_ptr(), cap, 0.0, 752.0, 0.0, 480.0, INV_W, INV_H, 100, 0.9, 1,
        m.data_ptr(), nm.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    n_h, mono_h, desc_h = n.cpu().numpy(), mono.cpu().numpy(), desc.cpu().numpy()
    kps_h = kps.cpu()
    ur, dep, m, nm = ur.cpu().numpy(), dep.cpu().numpy(), m.cpu().numpy(), nm.cpu().numpy()
    # oracle: one extractor object per image (the stereo search reads both pyramids)
    refs = []
    for i in range(P):
        el, er = O.OracleExtractor(1200, 1.2, 8, 20, 7), O.OracleExtractor(1200, 1.2, 8, 20, 7)
        lo, ro = el(left[i], (0, 0)), er(right[i], (0, 0))
        for f, o in ((i, lo), (P + i, ro)):
            same_frame(orb.keypoints_from_device(kps_h[f, :n_h[f]]), desc_h[f, :n_h[f]], int(mono_h[f]), *o)
        rur, rdep = O.compute_stereo_matches(el, er, lo[0], lo[1], ro[0], ro[1], BASE, MBF)
        assert (rur >= 0).sum() > len(lo[0]) // 4
        np.testing.assert_array_equal(ur[i, :n_h[i]].view(np.uint32), rur.view(np.uint32))
        np.testing.assert_array_equal(dep[i, :n_h[i]].view(np.uint32), rdep.view(np.uint32))
        refs.append(lo)
    total = 0
    for t in range(P - 1):
        k1, d1, _ = refs[t]
        prev = np.stack([k1["x"], k1["y"]], 1)
        rnm, rm12, _ = O.search_for_initialization(frame(*refs[t][:2]), frame(*refs[t + 1][:2]), prev, 100, 0.9,
                                                   True)
        assert int(nm[t]) == rnm
        np.testing.assert_array_equal(m[t, :len(k1)], rm12)
        total += rnm
    assert total > 100 * (P - 1)


def test_monocular_init_extractor_5000(gpu_lib):
    """ORBextractor(5*1000) on 752x480 (Tracking.cc:601), then the
    initialization search between two consecutive frames (Tracking.cc:2459)."""
    seq = synth.sequence(752, 480, 3, config=2, start=500)
    ex = orb.ORBextractor(5000, 1.2, 8, 20, 7)
    ref = O.OracleExtractor(5000, 1.2, 8, 20, 7)
    outs = []
    for i, lap in enumerate([(0, 1000), (0, 1000), (100, 300)]):
        k, d, mono = ex(seq[i], None, lap)
        rk, rd, rm = ref(seq[i], lap)
        same_frame(k, d, mono, rk, rd, rm)
        assert len(k) > 3000
        outs.append((k, d))
    k1, d1 = outs[0]
    prev = np.stack([k1["x"], k1["y"]], 1)
    nm, m12, prev_out = orb.ORBmatcher(0.9, True).SearchForInitialization(frame(k1, d1), frame(*outs[1]), prev, 100)
    rnm, rm12, rprev = O.search_for_initialization(frame(k1, d1), frame(*outs[1]), prev, 100, 0.9, True)
    assert nm == rnm and nm > 500
    np.testing.assert_array_equal(m12, rm12)
    np.testing.assert_array_equal(prev_out, rprev)


def test_monocular_init_over_8k_keypoints(gpu_lib):
    """The initialization search of Tracking's init extractor at nFeatures =
    2000 (ORBextractor(5 * 2000), Tracking.cc:601) on 1280x960 frames:
    > 8,192 keypoints a frame, beyond the LDS-resident pools of round 3 (the
    per-lane top-K from global memory and the 9-byte resolve state take it);
    matches and the updated vbPrevMatched equal the oracle's
    (ORBmatcher.cc:648-763)."""
    seq = synth.sequence(1280, 960, 2, config=2, start=700)
    ex = orb.ORBextractor(10000, 1.2, 8, 20, 7)
    outs = [ex(seq[i], None, (0, 1000))[:2] for i in range(2)]
    assert len(outs[0][0]) > 8192 and len(outs[1][0]) > 8192
    k1, d1 = outs[0]
    prev = np.stack([k1["x"], k1["y"]], 1)
    f1 = abi.frame_struct(k1, d1, 1280, 960)
    f2 = abi.frame_struct(*outs[1], 1280, 960)
    nm, m12, prev_out = orb.ORBmatcher(0.9, True).SearchForInitialization(f1, f2, prev, 100)
    rnm, rm12, rprev = O.search_for_initialization(f1, f2, prev, 100, 0.9, True)
    assert nm == rnm and nm > 1000
    np.testing.assert_array_equal(m12, rm12)
    np.testing.assert_array_equal(prev_out, rprev)


def test_monocular_init_extractor_5000_batch(gpu_lib):
    import torch
    seq = synth.sequence(752, 480, 6, config=2, start=700)
    ex = orb.ORBextractor(5000, 1.2, 8, 20, 7)
    kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
    torch.cuda.synchronize()
    ref = O.OracleExtractor(5000, 1.2, 8, 20, 7)
    for i in range(len(seq)):
        ni = int(n[i])
        same_frame(orb.keypoints_from_device(kps[i, :ni]), desc[i, :ni].cpu().numpy(), int(mono[i]),
                   *ref(seq[i], (0, 1000)))


@pytest.mark.parametrize("w,h,sf,nl", [(40, 30, 1.2, 1), (160, 120, 1.2, 9), (100, 300, 1.2, 1)])
def test_unsupported_size_fails_every_time(gpu_lib, w, h, sf, nl):
    """Sizes the reference does not survive are refused, every time: a level
    of <= 32 px on a side (DistributeOctTree divides by maxY - minY <= 0 and
    sizes a vector from it, ORBextractor.cc:559-565), and nIni = 0 with FAST
    cells (vpIniNodes[0] of an empty vector, :583-584).  A refused plan must
    not leave a plan behind that a second call with the same size takes for a
    built one, and the handle still works for a supported size afterwards."""
    ex = orb.ORBextractor(1000, sf, nl, 20, 7)
    img = synth.image(w, h, 5)
    assert O.OracleExtractor(1000, sf, nl, 20, 7).run_rc(img, (0, 1000)) < 0     # the oracle refuses too
    for _ in range(3):
        with pytest.raises(RuntimeError):
            ex(img, None, (0, 1000))
        assert capi.lib().orbx_max_keypoints(ex._h, w, h) < 0
    good = synth.image(752, 480, 6)
    same_frame(*ex(good, None, (0, 1000)), *O.OracleExtractor(1000, sf, nl, 20, 7)(good, (0, 1000)))


@pytest.mark.parametrize("w,h,sf,nl", [(160, 120, 1.2, 8), (752, 480, 2.0, 3), (640, 480, 2.0, 4),
                                        (120, 90, 1.2, 3)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_small_levels_and_exact_2x(gpu_lib, w, h, sf, nl, mode):
    """Sizes the reference accepts at the edges of the plan: levels of 33..66
    px (no FAST cells, ORBextractor.cc:798-799: no keypoints there) and exact
    2x reductions, where cv::resize takes INTER_AREA (resize.cpp:
    is_area_fast), whose 2x2 fast path (a + b + c + d + 2) >> 2 the linear
    fixed point reproduces.  Single image and a batch (mode 0 single-image
    path; 1 row bands, 2 sliding frame on 3 frames): keypoints, descriptors
    and every level equal the oracle's, and every exact-2x level equals the
    2x2 block average of the level above it."""
    import torch
    ex = orb.ORBextractor(1000, sf, nl, 20, 7)
    seq = synth.sequence(w, h, 3, config=2, start=400)
    if mode == 0:
        outs = [ex(seq[0], None, (0, 1000))]
        pyr = [ex.mvImagePyramid]
    else:
        ex.set_pyramid_mode(mode)
        kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
        torch.cuda.synchronize()
        outs = [(orb.keypoints_from_device(kps[f, :int(n[f])]), desc[f, :int(n[f])].cpu().numpy(), int(mono[f]))
                for f in range(3)]
        pyr = [ex.batch_pyramid(f) for f in range(3)]
    for f, (k, d, m) in enumerate(outs):
        ref = O.OracleExtractor(1000, sf, nl, 20, 7)
        same_frame(k, d, m, *ref(seq[f], (0, 1000)))
        for lev in range(nl):
            np.testing.assert_array_equal(pyr[f][lev], ref.level(lev), err_msg=f"frame {f} level {lev}")
        for lev in range(1, nl):
            a, b = pyr[f][lev - 1].astype(np.int32), pyr[f][lev]
            if a.shape[0] == 2 * b.shape[0] and a.shape[1] == 2 * b.shape[1]:
                avg = (a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
                np.testing.assert_array_equal(b, avg.astype(np.uint8), err_msg=f"INTER_AREA level {lev}")


def test_mixed_lapping_batch_keeps_every_pyramid(gpu_lib):
    """orbx_extract_batch with runs of different lapping areas (fisheye
    vLapL != vLapR, Frame.cc:1059-1060): every frame's pyramid stays in its
    own slot (orbx_get_batch_level), and a batch ends the single-image state."""
    l, r = synth.stereo_pair(752, 480, 3010)
    seq = synth.sequence(752, 480, 3, config=2, start=310)
    imgs = [l, r, seq[0], seq[1], seq[2]]
    laps = [(0, 500), (200, 751), (200, 751), (0, 1000), (0, 500)]
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    ex(synth.image(752, 480, 99), None, (0, 1000))          # a single-image call first
    out = ex.extract_batch(imgs, laps)
    for f, (im, lap, got) in enumerate(zip(imgs, laps, out)):
        ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
        same_frame(*got, *ref(im, lap))
        for lev, (a, b) in enumerate(zip(ex.batch_pyramid(f), [ref.level(x) for x in range(8)])):
            np.testing.assert_array_equal(a, b, err_msg=f"frame {f} level {lev}")
    with pytest.raises(RuntimeError):
        ex.mvImagePyramid                                    # noqa: B018  (no single image is current)
    ex(seq[0], None, (0, 1000))                               # single image again: batch state ends
    with pytest.raises(RuntimeError):
        ex.batch_pyramid(0)
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    ref(seq[0], (0, 1000))
    np.testing.assert_array_equal(ex.mvImagePyramid[3], ref.level(3))


def test_extract_batch_threaded_gather_row_steps(gpu_lib):
    """>= 32 frames (the multi-threaded pinned gather) given as views with a
    row step wider than the image; equal to one-image extraction."""
    nf = 40
    seq = synth.sequence(752, 480, nf, config=2, start=900)
    wide = np.zeros((nf, 480, 752 + 37), np.uint8)
    wide[:, :, 5:757] = seq
    views = [wide[i, :, 5:757] for i in range(nf)]
    assert views[0].strides[0] == 752 + 37
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    out = ex.extract_batch(views)
    single = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    for i in range(nf):
        same_frame(*out[i], *single(seq[i], None, (0, 1000)))
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    for i in (0, 17, 39):
        same_frame(*out[i], *ref(seq[i], (0, 1000)))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("w,h", [(752, 480), (753, 481), (756, 480), (1920, 1080), (320, 240)])
def test_pyramid_row_load_widths(gpu_lib, w, h, mode):
    """k_pyramid / k_pyr_stream stage level 0 with 16-byte, 4-byte or 1-byte
    row loads by the alignment of the caller's frames (row step = width here):
    every level of every frame equal to the oracle's ComputePyramid, keypoints
    too.  mode: 1 row bands, 2 sliding frame (forced on 3 frames)."""
    import torch
    seq = synth.sequence(w, h, 3, config=2, start=1200)
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    ex.set_pyramid_mode(mode)
    kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
    torch.cuda.synchronize()
    ran = ex.pyramid_kernel()
    if mode == 2 and (w, h) != (1920, 1080):
        assert ran == 2, "k_pyr_stream must take every size up to 756 px wide"
    else:
        assert ran in (mode, 1), ran
    for f in range(len(seq)):
        ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
        rk, rd, rm = ref(seq[f], (0, 1000))
        for lev, a in enumerate(ex.batch_pyramid(f)):
            np.testing.assert_array_equal(a, ref.level(lev), err_msg=f"frame {f} level {lev}")
        ni = int(n[f])
        same_frame(orb.keypoints_from_device(kps[f, :ni]), desc[f, :ni].cpu().numpy(), int(mono[f]), rk, rd, rm)


@pytest.mark.parametrize("w,h", [(752, 480), (320, 240), (512, 512)])
def test_pyr_stream_counters_at_lds_top(gpu_lib, w, h):
    """Round 2 moved k_pyr_stream's per-step wave-item counters from the top of
    its ~139 KiB LDS allocation to dword 0 after wrong pyramids and a hang,
    and blamed LDS atomics at high addresses.  With ORB_OPT_PYR_CNT_END the
    counters sit after the rings again -- outside the copied table image, so
    the kernel zeroes them -- and every level of every frame must still equal
    the oracle's ComputePyramid (ORBextractor.cc:1170-1195): the atomics at the
    top of LDS are fine once the counters start at zero."""
    import torch
    seq = synth.sequence(w, h, 40, config=2, start=1500)
    with capi.debug_option(capi.ORB_OPT_PYR_CNT_END, 1):     # read when the handle builds its plan
        ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
        ex.set_pyramid_mode(2)
        kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
        torch.cuda.synchronize()
    assert ex.pyramid_kernel() == 2
    for f in (0, 1, 17, 39):
        ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
        rk, rd, rm = ref(seq[f], (0, 1000))
        for lev, a in enumerate(ex.batch_pyramid(f)):
            np.testing.assert_array_equal(a, ref.level(lev), err_msg=f"frame {f} level {lev}")
        ni = int(n[f])
        same_frame(orb.keypoints_from_device(kps[f, :ni]), desc[f, :ni].cpu().numpy(), int(mono[f]), rk, rd, rm)


def _compass_candidates(img, t):
    """The compass pre-test of k_fast_cells / k_pyr_stream restated in numpy:
    every 9-arc of FAST's 16-ring holds one of {U, D} and one of {L, R}
    (the pixels 3 px away), so a corner at t has min(max(U,D), max(L,R)) > v + t
    (brighter ring) or max(min(U,D), min(L,R)) < v - t (darker ring)."""
    a = img.astype(np.int32)
    v = a[3:-3, 3:-3]
    U, D, Lf, R = a[:-6, 3:-3], a[6:, 3:-3], a[3:-3, :-6], a[3:-3, 6:]
    bright = np.minimum(np.maximum(U, D), np.maximum(Lf, R)) > v + t
    dark = np.maximum(np.minimum(U, D), np.minimum(Lf, R)) < v - t
    out = np.zeros(a.shape, bool)
    out[3:-3, 3:-3] = bright | dark
    return out


@pytest.mark.parametrize("w,h,ini,mn", [(752, 480, 20, 7), (512, 512, 20, 7), (640, 480, 12, 5), (320, 240, 20, 7),
                                        (753, 481, 30, 10)])
def test_fused_pretest_bitmap(gpu_lib, w, h, ini, mn):
    """k_pyr_stream's fused FAST pre-test (ORBextractor.cc:826 FAST(iniThFAST)
    candidates, computed while each level's rows sit in the LDS rings) equals
    the numpy compass test on the oracle's pyramid for every pixel of every
    level's window union, and the FAST pass that takes its candidates from it
    gives the oracle's keypoints and descriptors (ORBextractor.cc:781-896)."""
    import torch
    seq = synth.sequence(w, h, 3, config=2, start=900)
    with capi.debug_option(capi.ORB_OPT_PYR_PRETEST, 1):      # read when the handle builds its plan
        ex = orb.ORBextractor(1000, 1.2, 8, ini, mn)
        ex.set_pyramid_mode(2)
        kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
        torch.cuda.synchronize()
    assert ex.pyramid_kernel() == 2 and ex.plan_info(w, h)["pretest"] == 1
    for f in range(len(seq)):
        ref = O.OracleExtractor(1000, 1.2, 8, ini, mn)
        rk, rd, rm = ref(seq[f], (0, 1000))
        for lev in range(8):
            bm, (y0, y1, x0, x1) = ex.debug_pretest(f, lev)
            lv = ref.level(lev)
            want = _compass_candidates(lv, ini)
            got = bm[:lv.shape[0], :lv.shape[1]]
            np.testing.assert_array_equal(got[y0:y1, x0:x1], want[y0:y1, x0:x1], err_msg=f"frame {f} level {lev}")
        ni = int(n[f])
        same_frame(orb.keypoints_from_device(kps[f, :ni]), desc[f, :ni].cpu().numpy(), int(mono[f]), rk, rd, rm)
