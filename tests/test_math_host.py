"""Host checks of the product's scalar ports (csrc/orb_math.h compiled for
the CPU): glibc sincosf exhaustively over every float in [0, 2*pi], the
libstdc++ introsort port against std::sort, fastAtan2 against the oracle."""
import ctypes as C
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

SRC = Path(__file__).resolve().parent / "native" / "math_host_check.cpp"


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("mh") / "mathcheck.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so), str(SRC),
                    "-lpthread"], check=True)
    L = C.CDLL(str(so))
    L.sincos_mismatches.restype = C.c_longlong
    L.sincos_mismatches.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]
    L.sort_mismatches.argtypes = [C.c_int, C.c_int, C.c_uint]
    L.level_fallbacks.argtypes = []
    L.port_fast_atan2.restype = C.c_float
    L.port_fast_atan2.argtypes = [C.c_float, C.c_float]
    return L


def test_sincosf_exhaustive_0_2pi(lib):
    hi = struct.unpack("<I", struct.pack("<f", 6.2832))[0]   # just above 2*pi
    first = C.c_uint32(0)
    assert lib.sincos_mismatches(0, hi, 8, C.byref(first)) == 0, hex(first.value)


def test_introsort_port_matches_std_sort(lib):
    """The iterative port and the data-parallel restatement (partition by
    ranks, stable per-leaf insertion) both give std::sort's permutation."""
    assert lib.sort_mismatches(5000, 600, 7) == 0
    assert lib.sort_mismatches(2000, 40, 11) == 0
    assert lib.sort_mismatches(3000, 1200, 13) == 0
    assert lib.level_fallbacks() < 50


def test_fast_atan2_port_matches_oracle(lib):
    rng = np.random.default_rng(0)
    vals = rng.integers(-2_000_000, 2_000_000, size=(20000, 2)).astype(np.float32)
    vals[:50] = 0
    vals[50:100, 0] = 0
    for y, x in vals:
        assert lib.port_fast_atan2(float(y), float(x)) == O.fast_atan2(float(y), float(x))


def test_host_sort_statement_on_adversarial_inputs(lib):
    """McIlroy's quicksort adversary against libstdc++ std::sort reaches the
    introsort depth limit; the data-parallel statement reports it (so the
    device falls back to the sequential port, tests/test_gpu_sort.py)."""
    lib.antiqsort_vals.argtypes = [C.c_int, C.c_void_p]
    lib.levels_complete.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    for n in [40, 300, 2000]:
        v = np.zeros(n, np.int32)
        lib.antiqsort_vals(n, v.ctypes.data)
        assert sorted(v.tolist()) == list(range(n))
        z = np.zeros(n, np.int32)
        assert lib.levels_complete(n, v.ctypes.data, z.ctypes.data) == 0
        r = np.random.default_rng(n).permutation(n).astype(np.int32)
        assert lib.levels_complete(n, r.ctypes.data, z.ctypes.data) == 1
