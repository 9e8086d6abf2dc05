"""Exhaustive check of the DEVICE compile of k_describe's scalar math
(reference ORBextractor.cc:76-146): the product's
glibc_sincosf port, the degree->radian conversion with the 512 fused rBRIEF
sampling offsets, and fastAtan2, each evaluated on the GPU over its whole
input domain (orbx_debug_math) and compared chunk by chunk with the oracle
on the host, which calls the system libm's sincosf exactly like the
reference binary (orbo_debug_math, oracle/orb_oracle.cpp).  The host side
runs the oracle's -O3 -march build for this host's ISA level."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import capi

pytestmark = pytest.mark.gpu
LOG2 = 16


def fbits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def compare(what, begin, end, fused=1):
    n = ((end - begin) + (1 << LOG2) - 1) >> LOG2
    dev = np.zeros(n, np.uint64)
    host = np.zeros(n, np.uint64)
    rc = capi.lib().orbx_debug_math(0, what, begin, end, LOG2, fused, dev.ctypes.data)
    assert rc == 0, rc
    assert O.fast_lib().orbo_debug_math(what, begin, end, LOG2, fused, threads(), host.ctypes.data) == 0
    bad = np.nonzero(dev != host)[0]
    assert len(bad) == 0, f"{len(bad)} of {n} chunks differ, first elements {[begin + (int(b) << LOG2) for b in bad[:4]]}"
    return n


def test_sincosf_every_float_0_2pi(gpu_lib):
    """every float bit pattern in [0, 6.2832] (radians): the device port vs libm"""
    assert compare(0, 0, fbits(6.2832) + 1) > 16000


def test_sampling_offsets_every_degree_angle(gpu_lib):
    """every float angle in [0, 360] degrees (fastAtan2's range): angle
    conversion, sincosf, and cvRound(fmaf(x, b, y*a)), cvRound(fmaf(x, a, -(y*b)))
    for all 512 pattern points (ORBextractor.cc:110-118)"""
    assert compare(1, 0, fbits(360.0) + 1, fused=1) > 17000


def test_sampling_offsets_unfused_sample(gpu_lib):
    """the unfused form (fma_sampling=0 knob) on [1, 2) degrees and [180, 181)"""
    compare(1, fbits(1.0), fbits(2.0), fused=0)
    compare(1, fbits(180.0), fbits(181.0), fused=0)


def test_fast_atan2_moment_pairs(gpu_lib):
    """every integer pair in [-2048, 2048]^2 plus 2^26 pseudo-random pairs over
    +-1.5e6 (the range of IC_Angle's moments)"""
    compare(2, 0, 4097 * 4097 + (1 << 26))


def test_debug_math_arguments(gpu_lib):
    h = np.zeros(4, np.uint64)
    assert capi.lib().orbx_debug_math(0, 3, 0, 100, LOG2, 1, h.ctypes.data) != 0
    assert capi.lib().orbx_debug_math(0, 0, 10, 5, LOG2, 1, h.ctypes.data) != 0
    assert capi.lib().orbx_debug_math(0, 0, 0, 1 << 33, LOG2, 1, None) != 0
