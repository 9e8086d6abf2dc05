"""Vocabulary side, host code of the product library:
the DBoW2 text loader, BowVector/FeatureVector assembly and the six scores,
against the independent restatements in tests/vocab_ref.py.  No GPU."""
import numpy as np
import pytest

from orb_slam3_vio_fixes_amd import orb, synth
from tests import vocab_ref as R


def tree(k, L, seed):
    v = synth.vocabulary(k, L, seed)
    v["child_idx"] = None
    return v


def same_vocab(lib: orb.TextVocabulary, ref: dict):
    a = lib.arrays()
    assert (lib.k, lib.L, lib.scoring, lib.weighting, lib.nwords) == \
        (ref["k"], ref["depth_levels"], ref["scoring"], ref["weighting"], ref["nwords"])
    for key in ("first_child", "nchild", "child_idx", "node_desc", "word_id"):
        np.testing.assert_array_equal(a[key], ref[key], err_msg=key)
    np.testing.assert_array_equal(a["weight"].view(np.uint64), ref["weight"].view(np.uint64))


@pytest.mark.parametrize("k,L,seed,trailing", [(5, 3, 1, True), (5, 3, 1, False), (10, 4, 2, True), (3, 5, 3, True)])
def test_text_loader_round_trip(tmp_path, k, L, seed, trailing):
    v = tree(k, L, seed)
    path = tmp_path / "voc.txt"
    R.save_text(path, v, k, 0, 0, trailing_newline=trailing)
    ref = R.load_text(path)
    lib = orb.TextVocabulary(path)
    same_vocab(lib, ref)
    n_written = v["nnodes"]
    # the reference's empty read after a final newline adds one root child
    assert lib.nnodes == n_written + (1 if trailing else 0)
    assert lib.nwords == k ** L
    if trailing:
        a = lib.arrays()
        assert a["child_idx"][a["first_child"][0] + a["nchild"][0] - 1] == n_written
    # descriptors and words of the written nodes survive the round trip
    np.testing.assert_array_equal(lib.arrays()["node_desc"][1:n_written], v["node_desc"][1:])


@pytest.mark.parametrize("text", ["10 6 0 0", "10 6 0 0\n", "10 6 0 0\n0 1 " + "7 " * 32 + " 0.5\n\n0 1 " + "9 " * 32 +
                                  " 0.25", "10 6 1 2\n0 1 1 2 3\n", "10 6 0 0\r\n0 1 " + "1 " * 32 + " 1e-3\r\n"])
def test_text_loader_edge_cases(tmp_path, text):
    path = tmp_path / "voc.txt"
    path.write_bytes(text.encode())
    same_vocab(orb.TextVocabulary(path), R.load_text(path))


@pytest.mark.parametrize("text", ["", "21 6 0 0\n", "10 0 0 0\n", "10 6 6 0\n", "abc\n", "10 6 0 0\n5 1 2\n"])
def test_text_loader_rejects(tmp_path, text):
    path = tmp_path / "voc.txt"
    path.write_bytes(text.encode())
    with pytest.raises(ValueError):
        orb.TextVocabulary(path)


def test_text_loader_missing_file(tmp_path):
    with pytest.raises(ValueError):
        orb.TextVocabulary(tmp_path / "nope.txt")


@pytest.mark.parametrize("scoring", range(6))
@pytest.mark.parametrize("weighting", range(4))
def test_bow_assembly(scoring, weighting):
    from orb_slam3_vio_fixes_amd import abi, capi
    import ctypes as C
    rng = np.random.default_rng(scoring * 10 + weighting)
    n = 700
    wid = rng.integers(0, 300, n).astype(np.int32)
    w = rng.uniform(0, 3, n)
    w[rng.random(n) < 0.1] = 0.0                        # stopped words
    nid = rng.integers(0, 60, n).astype(np.int32)
    bw, bv = np.zeros(n, np.int32), np.zeros(n)
    fn, fo, fi = np.zeros(n, np.int32), np.zeros(n + 1, np.int32), np.zeros(n, np.int32)
    nb, nf = C.c_int32(), C.c_int32()
    capi.check(capi.lib().orbv_bow_assemble(scoring, weighting, n, abi.ptr(wid), abi.ptr(w), abi.ptr(nid),
                                            abi.ptr(bw), abi.ptr(bv), C.byref(nb), abi.ptr(fn), abi.ptr(fo),
                                            abi.ptr(fi), C.byref(nf)), "assemble")
    rw, rv, rfv = R.bow_assemble(scoring, weighting, wid, w, nid)
    np.testing.assert_array_equal(bw[:nb.value], rw)
    np.testing.assert_array_equal(bv[:nb.value].view(np.uint64), rv.view(np.uint64))
    assert list(fn[:nf.value]) == list(rfv)
    for j, node in enumerate(rfv):
        assert list(fi[fo[j]:fo[j + 1]]) == rfv[node]


@pytest.mark.parametrize("scoring", range(6))
def test_scores(scoring):
    rng = np.random.default_rng(100 + scoring)
    for trial in range(20):
        w1 = np.unique(rng.integers(0, 400, rng.integers(1, 200))).astype(np.int32)
        w2 = np.unique(np.concatenate([rng.choice(w1, len(w1) // 2), rng.integers(0, 400, 50)])).astype(np.int32)
        v1 = rng.uniform(0.01, 1, len(w1))
        v2 = rng.uniform(0.01, 1, len(w2))
        v1 /= v1.sum()
        v2 /= v2.sum()
        got = orb.score(scoring, w1, v1, w2, v2)
        assert np.float64(got).view(np.uint64) == np.float64(R.score(scoring, w1, v1, w2, v2)).view(np.uint64)
