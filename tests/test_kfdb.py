"""DetectRelocalizationCandidates: the oracle against
the independent Python restatement (CPU), and the GPU path against the oracle
on keyframe databases up to 10,000 keyframes, including the stale
mRelocScore the reference reads for unscored neighbours."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import kfdb_ref as R


@pytest.mark.parametrize("nkf,nwords,seed", [(60, 500, 1), (300, 2000, 2), (1000, 5000, 3)])
def test_oracle_reloc_vs_python(nkf, nwords, seed):
    db = R.make_db(nkf, nwords, seed)
    rng = np.random.default_rng(seed)
    stale = rng.uniform(0, 0.3, nkf).astype(np.float32)
    nonempty = 0
    for q in range(6):
        qw, qv = R.make_query(db, seed * 100 + q)
        for map_id in (0, 1):
            a, b = stale.copy(), stale.copy()
            got = O.detect_relocalization_candidates(db, qw, qv, map_id, a)
            ref = R.detect(db, qw, qv, map_id, b)
            assert list(got) == ref
            np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
            nonempty += len(ref) > 0
    assert nonempty >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("nkf,nwords,seed", [(300, 2000, 2), (2000, 20000, 4), (10000, 100000, 5)])
def test_gpu_reloc_vs_oracle(gpu_lib, nkf, nwords, seed):
    from orb_slam3_vio_fixes_amd import orb
    db = R.make_db(nkf, nwords, seed)
    gdb = orb.KeyFrameDatabase(db)
    rng = np.random.default_rng(seed)
    a = rng.uniform(0, 0.3, nkf).astype(np.float32)
    b = a.copy()
    for q in range(8):                          # stale scores carry over between queries
        qw, qv = R.make_query(db, seed * 100 + q)
        map_id = q % 2
        got = gdb.DetectRelocalizationCandidates(qw, qv, map_id, a)
        ref = O.detect_relocalization_candidates(db, qw, qv, map_id, b)
        assert list(got) == list(ref)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
