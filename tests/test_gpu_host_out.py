"""The single-launch host calls in their other result modes (ORB_OPT_HOST_OUT
1: zero-copy block + stream sync; 2: device block copied back) equal the
oracle, as the default (zero-copy block + completion word) does
(tests/test_gpu_matcher.py)."""
import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, capi, orb, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames():
    seq = synth.sequence(752, 480, 3, config=11)
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    return [ex(seq[i], (0, 1000)) for i in range(3)]


def fr(f):
    return abi.frame_struct(f[0], f[1], 752, 480, scale_factors=np.float32(1.2) ** np.arange(8, dtype=np.float32))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("sfi", ["fused", "grid"])
def test_initialization_result_modes(gpu_lib, frames, debug_option, sfi_form, sfi, mode):
    debug_option(capi.ORB_OPT_HOST_OUT, mode)
    sfi_form(sfi)
    for i1, i2 in [(0, 1), (1, 2)]:
        f1, f2 = frames[i1], frames[i2]
        prev = np.stack([f1[0]["x"], f1[0]["y"]], 1)
        nm, m12, p2 = orb.ORBmatcher(0.9, True).SearchForInitialization(fr(f1), fr(f2), prev, 100)
        rnm, rm12, rp2 = O.search_for_initialization(fr(f1), fr(f2), prev, 100, 0.9, True)
        assert nm == rnm
        np.testing.assert_array_equal(m12, rm12)
        np.testing.assert_array_equal(p2, rp2)


@pytest.mark.parametrize("mode", [1, 2])
def test_bow_result_modes(gpu_lib, frames, debug_option, mode):
    debug_option(capi.ORB_OPT_HOST_OUT, mode)
    rng = np.random.default_rng(5)
    f1, f2 = frames[0], frames[1]
    n1, n2 = len(f1[0]), len(f2[0])
    node1 = rng.integers(0, 40, n1)
    node2 = rng.integers(0, 40, n2)
    valid = (rng.random(n1) < 0.9).astype(np.uint8)
    kfv, fv = abi.featvec_struct(node1), abi.featvec_struct(node2)
    nm, match = orb.ORBmatcher(0.7, True).SearchByBoW(fr(f1), kfv, valid, fr(f2), fv)
    rnm, rmatch = O.search_by_bow(fr(f1), kfv, valid, fr(f2), fv, 0.7, True)
    assert nm == rnm
    np.testing.assert_array_equal(match, rmatch)


@pytest.mark.parametrize("upload", [0, 1])
def test_projection_upload_forms(gpu_lib, frames, debug_option, upload):
    """Inputs uploaded by the pull kernel (ORB_OPT_UPLOAD 0, default) or by
    hipMemcpyAsync (1): the same owners as the oracle."""
    debug_option(capi.ORB_OPT_UPLOAD, upload)
    rng = np.random.default_rng(11 + upload)
    src, cur = frames[0], frames[1]
    k = src[0][:500]
    qx = (k["x"] + rng.normal(0, 3, len(k)) + 3).astype(np.float32)
    qy = (k["y"] + rng.normal(0, 3, len(k)) + 3).astype(np.float32)
    n = len(k)
    mps = abi.mappoints_struct(qx, qy, qx - rng.uniform(0, 40, n).astype(np.float32), k["octave"],
                               rng.uniform(0.99, 1.0, n).astype(np.float32), rng.uniform(0, 100, n).astype(np.float32),
                               (rng.random(n) < 0.9).astype(np.uint8), (rng.random(n) < 0.7).astype(np.uint8),
                               src[1][:n])
    N = len(cur[0])
    F = fr(cur)
    owner = np.full(N, -1, np.int32)
    blocked = np.zeros(N, np.uint8)
    nm, own = orb.ORBmatcher(0.8, True).SearchByProjection(F, mps, 3.0, False, 50.0, owner, blocked)
    rnm, rown = O.search_by_projection_mps(F, mps, 3.0, False, 50.0, 0.8, owner, blocked)
    assert nm == rnm and nm > 0
    np.testing.assert_array_equal(own, rown)
