"""DistributeOctTree forms on the GPU against the CPU oracle
(ORBextractor.cc:555-779): the 4-wave k_quadtree for every level (the
default), the one-wave k_quadtree_w (ORB_OPT_QT_FORM 1: keys in registers,
levels of more than 1,536 keys flagged and left to k_quadtree in a fixup
launch), and the one-wave form with a small key capacity (ORB_OPT_QT_FORM 2 +
kcap) so that some or all levels of a frame take the fixup path beside levels
distributed by the wave.  Every keypoint byte, descriptor and monoIndex is compared, in
single-image calls and in batches (the per-(frame, level) overflow flags of
one launch are mixed)."""

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import capi, orb, synth

pytestmark = pytest.mark.gpu

# ORB_OPT_QT_FORM values: 4-wave form (default), one-wave form, one-wave with
# key capacity 0, 300 (levels 0-3 of a C2 frame overflow, 4-7 do not) and 700
FORMS = {"block": 0, "wave": 1, "kcap0": 2, "kcap300": 302, "kcap700": 702}


def same(k, d, m, rk, rd, rm, what=""):
    assert (len(k), m) == (len(rk), rm), what
    assert np.array_equal(k.view(np.uint8), rk.view(np.uint8)), f"keypoints differ {what}"
    assert np.array_equal(d, rd), f"descriptors differ {what}"


@pytest.mark.parametrize("form", list(FORMS))
def test_quadtree_forms_single_image(gpu_lib, debug_option, form):
    debug_option(capi.ORB_OPT_QT_FORM, FORMS[form])
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    for i, img in enumerate(synth.sequence(752, 480, 3, config=2, start=7)):
        same(*ex(img, None, (0, 1000)), *ref(img, (0, 1000)), what=f"frame {i}")


@pytest.mark.parametrize("form", ["block", "wave", "kcap300", "kcap700"])
def test_quadtree_forms_batch(gpu_lib, debug_option, form):
    import torch
    debug_option(capi.ORB_OPT_QT_FORM, FORMS[form])
    B = 24
    seq = synth.sequence(752, 480, B, config=2, start=300)
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    kps, desc, n, mono, cap = ex.extract_batch_device(torch.from_numpy(seq).cuda(), (0, 1000))
    torch.cuda.synchronize()
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    for f in range(0, B, 5):
        k = orb.keypoints_from_device(kps[f, :int(n[f])])
        same(k, desc[f, :int(n[f])].cpu().numpy(), int(mono[f]), *ref(seq[f], (0, 1000)), what=f"frame {f}")


def test_quadtree_dense_level_overflows_to_block_form(gpu_lib, debug_option):
    """A noise image of 1920x1080 at nFeatures 1000: its levels 0-6 hold far
    more than 1,536 FAST keys (the one-wave capacity), so they go through the
    overflow flag to k_quadtree while level 7 stays in the wave."""
    debug_option(capi.ORB_OPT_QT_FORM, FORMS["wave"])
    img = np.random.default_rng(5).integers(0, 256, (1080, 1920), dtype=np.uint8)
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    rk, rd, rm = ref(img, (0, 1000))
    stage0 = ref.stage(0, cap=4_000_000)
    assert len(stage0[0]) > 1536 and len(stage0[-1]) < 1536, [len(s) for s in stage0]
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    same(*ex(img, None, (0, 1000)), rk, rd, rm)


@pytest.mark.parametrize("nl,sf,nf", [(8, 1.2, 500), (4, 1.5, 2000), (1, 1.2, 300), (8, 1.2, 3000)])
def test_quadtree_wave_parameters(gpu_lib, debug_option, nl, sf, nf):
    """Level counts, scale factors and feature counts that move N, nIni and the
    number of last rounds (nf 3000: nodes beyond the wave's 64-node chunks)."""
    debug_option(capi.ORB_OPT_QT_FORM, FORMS["wave"])
    ex = orb.ORBextractor(nf, sf, nl, 20, 7)
    ref = O.OracleExtractor(nf, sf, nl, 20, 7)
    for seed in (11, 12):
        img = synth.image(752, 480, seed)
        same(*ex(img, None, (0, 1000)), *ref(img, (0, 1000)), what=f"seed {seed}")


@pytest.mark.parametrize("form", ["block", "wave"])
def test_quadtree_wide_frame_many_initial_nodes(gpu_lib, debug_option, form):
    """A 1600x200 frame: nIni = round(W / H) initial nodes per level (up to 11
    at level 0), several of them empty on a frame with a blank band."""
    debug_option(capi.ORB_OPT_QT_FORM, FORMS[form])
    img = synth.image(1600, 200, 21)
    img[:, 300:700] = 90
    ex = orb.ORBextractor(1000, 1.2, 4, 20, 7)
    ref = O.OracleExtractor(1000, 1.2, 4, 20, 7)
    same(*ex(img, None, (0, 1000)), *ref(img, (0, 1000)))
