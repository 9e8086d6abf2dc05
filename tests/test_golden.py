"""The oracle against its committed regression fixtures (tests/golden/),
including the SHA-256 of every regenerated synthetic input."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, synth

G = Path(__file__).resolve().parent / "golden"
MAN = json.loads((G / "manifest.json").read_text())


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: f"{c['name']}-{c['seed']}")
def test_oracle_matches_fixture(case):
    img = synth.image(case["w"], case["h"], case["seed"])
    assert sha(img) == case["image_sha"], "synthetic generator drifted"
    ex = O.OracleExtractor(case["nfeatures"], 1.2, 8, 20, 7)
    k, d, m = ex(img, tuple(case["lapping"]))
    assert (len(k), m) == (case["n"], case["mono"])
    assert sha(k) == case["kps_sha"] and sha(d) == case["desc_sha"]


def test_sequence_fixture_and_sfi():
    z = np.load(G / "c2_sequence01.npz")
    seq = synth.sequence(752, 480, 2, config=2, start=0)
    info = MAN["sfi_c2_sequence_0_1"]
    assert sha(seq[0]) == info["image0_sha"] and sha(seq[1]) == info["image1_sha"]
    ex = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    k0, d0, m0 = ex(seq[0], (0, 1000))
    k1, d1, _ = ex(seq[1], (0, 1000))
    assert np.array_equal(k0.view(np.uint8), z["kps"]) and np.array_equal(d0, z["desc"])
    prev = np.stack([k0["x"], k0["y"]], 1)
    nm, m12, prev2 = O.search_for_initialization(abi.frame_struct(k0, d0, 752, 480), abi.frame_struct(k1, d1, 752, 480),
                                                 prev, 100, 0.9, True)
    assert nm == info["nmatches"] == int(z["sfi_n"])
    np.testing.assert_array_equal(m12, z["sfi_matches"])
    np.testing.assert_array_equal(prev2, z["sfi_prev"])
