"""The device std::sort emulation of k_quadtree, pinned directly (SURVEY.md
A.3): DistributeOctTree's last rounds sort (count, node) pairs with
std::sort under compareNodes (reference src/ORBextractor.cc:538-553, :700),
an UNSTABLE libstdc++ introsort whose tie order decides which nodes expand
first.  The kernel restates it with ballot-built partition lists per wave
and per-leaf insertion sorts (block_std_sort, csrc/extractor.hip), with the
sequential port at the depth limit.  orbx_debug_sort runs exactly that code
on the GPU; the expected permutations come from the host's own std::sort on
pair<int, Node*> with the reference's comparator (tests/native/
math_host_check.cpp).  Inputs: heavy (count, UL.x) ties, n from 2 to 4000,
and McIlroy's quicksort adversary, which drives introsort to its depth limit."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

from orb_slam3_vio_fixes_amd import capi

pytestmark = pytest.mark.gpu
SRC = Path(__file__).resolve().parent / "native" / "math_host_check.cpp"


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    so = tmp_path_factory.mktemp("srt") / "mathcheck.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so), str(SRC),
                    "-lpthread"], check=True)
    L = C.CDLL(str(so))
    L.std_sort_perm.argtypes = [C.c_int] + [C.c_void_p] * 4
    L.antiqsort_vals.argtypes = [C.c_int, C.c_void_p]
    L.levels_complete.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    return L


def _p(a):
    return C.c_void_p(a.ctypes.data)


def run_both(host, arrays):
    """(device perm, host std::sort perm, device fallback flags) of a list
    of (cnt, x0) int32 array pairs."""
    off = np.zeros(len(arrays) + 1, np.int32)
    off[1:] = np.cumsum([len(c) for c, _ in arrays])
    cnt = np.ascontiguousarray(np.concatenate([c for c, _ in arrays]).astype(np.int32))
    x0 = np.ascontiguousarray(np.concatenate([x for _, x in arrays]).astype(np.int32))
    dev = np.full(len(cnt), -1, np.int32)
    fb = np.full(len(arrays), -1, np.int32)
    rc = capi.lib().orbx_debug_sort(0, len(arrays), _p(off), _p(cnt), _p(x0), _p(dev), _p(fb))
    assert rc == 0, rc
    ref = np.zeros(len(cnt), np.int32)
    host.std_sort_perm(len(arrays), _p(off), _p(cnt), _p(x0), _p(ref))
    return dev, ref, fb, off


def tied_arrays(rng, count, nmin, nmax):
    out = []
    for _ in range(count):
        n = int(rng.integers(nmin, nmax + 1))
        cmax, xmax = int(rng.integers(1, 7)), int(rng.integers(1, 9))
        out.append((2 + rng.integers(0, cmax, n), rng.integers(0, xmax, n)))
    return out


@pytest.mark.parametrize("seed,count,nmin,nmax", [(1, 60000, 2, 64), (2, 30000, 17, 300), (3, 10000, 300, 2000),
                                                  (4, 600, 2000, 4000)])
def test_device_sort_heavy_ties(gpu_lib, host, seed, count, nmin, nmax):
    """>= 10^5 arrays in all: counts in 2..7 and UL.x in 0..7, so nearly
    every comparison is a tie the unstable sort resolves by its own order."""
    rng = np.random.default_rng(seed)
    dev, ref, fb, off = run_both(host, tied_arrays(rng, count, nmin, nmax))
    bad = np.nonzero(dev != ref)[0]
    assert len(bad) == 0, f"{len(bad)} positions differ, first in array {np.searchsorted(off, bad[0], 'right') - 1}"


def test_device_sort_depth_limit(gpu_lib, host):
    """McIlroy's adversary against libstdc++ std::sort: introsort reaches its
    depth limit (where libstdc++ heap-sorts); the device must detect it
    (fallback flag), rerun the array through the sequential port and still
    give std::sort's permutation.  Mixed with tie-heavy killer variants."""
    arrays, expect_fb = [], []
    for n in [40, 64, 100, 257, 500, 1000, 2000, 3000, 4000]:
        v = np.zeros(n, np.int32)
        host.antiqsort_vals(n, _p(v))
        z = np.zeros(n, np.int32)
        assert host.levels_complete(n, _p(v), _p(z)) == 0      # the host statement hits the limit too
        arrays.append((v, z))
        expect_fb.append(1)
        # the same order of values spread over (count, UL.x) pairs: x0 breaks count ties
        arrays.append((v // 7 + 2, v % 7))
        expect_fb.append(1)
    rng = np.random.default_rng(9)
    for n in rng.integers(17, 4000, 40):
        c, x = 2 + rng.integers(0, 5, n), rng.integers(0, 6, n)
        arrays.append((c, x))
        expect_fb.append(-1)                                      # either way
    dev, ref, fb, off = run_both(host, arrays)
    np.testing.assert_array_equal(dev, ref)
    for f, e in zip(fb, expect_fb):
        if e == 1:
            assert f == 1


def test_device_sort_small_and_sorted_inputs(gpu_lib, host):
    """Edge shapes: n = 0, 1, 2, 16, 17, already sorted, reversed, all equal."""
    arrays = [(np.zeros(0, np.int32), np.zeros(0, np.int32))]
    for n in [1, 2, 3, 15, 16, 17, 18, 33, 1000, 4000]:
        a = np.arange(n, dtype=np.int32)
        arrays += [(a + 2, np.zeros(n, np.int32)), (a[::-1] + 2, np.zeros(n, np.int32)),
                   (np.full(n, 5, np.int32), np.full(n, 3, np.int32)), (np.full(n, 5, np.int32), a[::-1].copy())]
    dev, ref, fb, off = run_both(host, arrays)
    np.testing.assert_array_equal(dev, ref)
