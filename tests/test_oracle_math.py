"""CPU checks of the oracle's host side of the exhaustive device math check
(orbo_debug_math, used by tests/test_gpu_math.py): the tiny-angle shortcut
equals the full evaluation, and the -O3 -march builds (bench.py's
cpu_baseline, the math check's host side) agree with the -O2 checker."""
import struct

import numpy as np
import pytest

from oracle import oracle as O

LOG2 = 12


def fbits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def hashes(L, what, b, e, fused):
    h = np.zeros(((e - b) + (1 << LOG2) - 1) >> LOG2, np.uint64)
    assert L.orbo_debug_math(what, b, e, LOG2, fused, 4, h.ctypes.data) == 0
    return h


@pytest.mark.parametrize("b", [0, 0x00800000, 0x1F000000, fbits(2.0 ** -36) - (1 << 14)])
@pytest.mark.parametrize("fused", [0, 1])
def test_tiny_angle_shortcut_equals_full_evaluation(b, fused):
    L = O.lib()
    e = b + (1 << 14)
    assert np.array_equal(hashes(L, 1, b, e, fused), hashes(L, 1, b, e, fused | 2))


@pytest.mark.parametrize("what,b,e", [(0, fbits(0.5), fbits(0.5) + (1 << 18)),
                                      (1, fbits(37.0), fbits(37.0) + (1 << 14)),
                                      (1, fbits(359.0), fbits(360.0) + 1),
                                      (2, 0, 1 << 18), (2, 4097 * 4097, 4097 * 4097 + (1 << 18))])
def test_march_builds_agree_with_checker(what, b, e):
    fast, _ = O.fast_variant()
    if fast == O.LIB:
        pytest.skip("no -march build for this host")
    assert np.array_equal(hashes(O.lib(), what, b, e, 1), hashes(O.lib(fast), what, b, e, 1))
