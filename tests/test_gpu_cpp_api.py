"""The C++ host interface (include/orb_slam3_mi355x.hpp) on the GPU: a
compiled program extracts and matches two frames; its hashes must equal the
oracle's outputs."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import abi, build, synth

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def fnv(b: bytes) -> str:
    h = 1469598103934665603
    for x in b:
        h ^= x
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def test_cpp_interface(gpu_lib, tmp_path):
    lib = build.build()
    exe = tmp_path / "cpp_api_test"
    subprocess.run(["g++", "-O2", "-std=c++17", str(ROOT / "tests/native/cpp_api_test.cpp"), "-o", str(exe),
                    str(lib), f"-Wl,-rpath,{lib.parent}"], check=True)
    seq = synth.sequence(752, 480, 2, config=13)
    for i in range(2):
        (tmp_path / f"im{i}.raw").write_bytes(seq[i].tobytes())
    out = subprocess.run([str(exe), str(tmp_path / "im0.raw"), str(tmp_path / "im1.raw"), "752", "480"],
                         check=True, capture_output=True, text=True).stdout.split()
    ref = O.OracleExtractor(1000, 1.2, 8, 20, 7)
    k0, d0, m0 = ref(seq[0], (0, 1000))
    k1, d1, m1 = ref(seq[1], (0, 1000))
    prev = np.stack([k0["x"], k0["y"]], 1)
    nm, m12, _ = O.search_for_initialization(abi.frame_struct(k0, d0, 752, 480), abi.frame_struct(k1, d1, 752, 480),
                                             prev, 100, 0.9, True)
    f0, f1 = abi.frame_struct(k0, d0, 752, 480), abi.frame_struct(k1, d1, 752, 480)
    fv0, fv1 = abi.featvec_struct(np.arange(len(k0)) % 16), abi.featvec_struct(np.arange(len(k1)) % 16)
    nb, b12 = O.search_by_bow_kf(f0, fv0, np.ones(len(k0), np.uint8), f1, fv1, np.ones(len(k1), np.uint8), 0.75,
                                 True)
    assert nb > 0
    assert out == [str(len(k0)), str(m0), fnv(k0.tobytes()), fnv(d0.tobytes()), str(len(k1)), str(m1), str(nm),
                   fnv(m12.astype(np.int32).tobytes()), str(nb), fnv(b12.astype(np.int32).tobytes())]
