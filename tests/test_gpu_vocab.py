"""GPU descent through a vocabulary loaded from the DBoW2 text format (node
ids = line numbers, explicit children lists, the reference's extra root child
after a final newline): word ids, weights and node ids equal the oracle's, and
the BowVector / FeatureVector assembled from them equal the Python
restatement of transform(features, v, fv, levelsup)."""
import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import orb, synth
from tests import vocab_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("trailing", [True, False])
def test_text_vocab_transform(gpu_lib, tmp_path, trailing):
    v = synth.vocabulary(10, 4, seed=77)
    v["child_idx"] = None
    path = tmp_path / "voc.txt"
    R.save_text(path, v, 10, 0, 0, trailing_newline=trailing)
    voc = orb.TextVocabulary(path)
    img = synth.image(1920, 1080, 5000)
    k, d, _ = orb.ORBextractor(5000, 1.2, 8, 20, 7)(img, None, (0, 1000))
    d = np.concatenate([d, np.zeros((3, 32), np.uint8)])          # all-zero rows: the extra root child's descriptor
    got = orb.transform(voc, d, 2)
    ref = O.transform(voc, d, 2)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    if trailing:
        assert (got[0][-3:] == 0).all() and (got[1][-3:] == 0).all()   # word 0, weight 0 (Node() defaults)
    bw, bv, fn, fo, fi = orb.transform_bow(voc, d, voc.scoring, voc.weighting, 2)
    rw, rv, rfv = R.bow_assemble(voc.scoring, voc.weighting, *ref)
    np.testing.assert_array_equal(bw, rw)
    np.testing.assert_array_equal(bv.view(np.uint64), rv.view(np.uint64))
    assert list(fn) == list(rfv)


def test_transform_device_resident_vocabulary(gpu_lib):
    """orbv_transform_device on a vocabulary held as CUDA tensors (the form a
    multi-GPU job keeps after its one RCCL broadcast, sharding.py) equals the
    host-API descent and the oracle, for a generated tree (implicit children)."""
    import torch
    from orb_slam3_vio_fixes_amd import abi, sharding
    vh = synth.vocabulary(10, 5, seed=91)
    vt = {k: torch.from_numpy(np.ascontiguousarray(vh[k])).cuda()
          for k in ("first_child", "nchild", "node_desc", "word_id", "weight")}
    vt.update(nnodes=int(vh["nnodes"]), depth_levels=int(vh["depth_levels"]), child_idx=None)
    img = synth.image(1920, 1080, 5001)
    _, d, _ = orb.ORBextractor(5000, 1.2, 8, 20, 7)(img, None, (0, 1000))
    got = orb.transform_device(sharding.vocab_device_struct(vt), torch.from_numpy(d).cuda(), 3)
    torch.cuda.synchronize()
    got = [x.cpu().numpy() for x in got]
    host = orb.transform(abi.vocab_struct(vh), d, 3)
    ref = O.transform(abi.vocab_struct(vh), d, 3)
    for a, b, c in zip(got, host, ref):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(a, c)
