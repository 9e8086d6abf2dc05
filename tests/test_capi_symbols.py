"""The product library loads without a GPU and exports every function the C
header declares (no compute calls)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "orb_mi355x.h"


def declared():
    txt = re.sub(r"/\*.*?\*/", " ", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(orb(?:[xmvsk]|_debug)_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("orbx_create", "orbx_extract", "orbx_extract_batch_device", "orbm_search_for_initialization",
                 "orbm_search_by_bow", "orbm_search_by_projection_mps", "orbm_search_by_projection_last",
                 "orbv_transform"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from orb_slam3_vio_fixes_amd import build, capi
    build.build()
    L = capi.load()
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    assert set(capi.EXPORTS) == set(declared())


def test_release_library_reads_no_environment():
    """Kernel choice is not switchable from a process's environment: the
    release library imports no getenv (alternative forms are reachable only
    through the explicit orb_debug_set_option test hook)."""
    import subprocess
    from orb_slam3_vio_fixes_amd import build, capi
    build.build()
    out = subprocess.run(["nm", "-D", "--undefined-only", str(capi.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "getenv" not in out
    L = capi.load()
    assert L.orb_debug_get_option(capi.ORB_OPT_PROJ_FORM) == 0
    assert L.orb_debug_set_option(99, 1) == -3 and L.orb_debug_get_option(99) == -1


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from orb_slam3_vio_fixes_amd import orb
    with pytest.raises(RuntimeError):
        orb.ORBextractor(1000, 1.2, 8, 20, 7)


def test_argument_checks_before_the_device():
    """Entry points reject bad arguments before touching a device (these run
    with no GPU): ORB_ERR_PARAM (-3); an empty candidate set is a no-op."""
    import ctypes as C
    from orb_slam3_vio_fixes_amd import capi
    L = capi.load()
    PARAM = -3
    assert L.orbm_search_by_bow_many(-1, None, None, None, None, None, 0.75, 1, None, None) == PARAM
    cnt = (C.c_int32 * 1)()
    match = (C.c_int32 * 1)()
    # nkf = 0 with a frame and its FeatureVector: nothing to do, ORB_OK
    import numpy as np
    from orb_slam3_vio_fixes_amd import abi
    k = np.zeros(1, abi.KEYPOINT_DTYPE)
    d = np.zeros((1, 32), np.uint8)
    F = abi.frame_struct(k, d, 64, 64)
    fv = abi.featvec_struct(np.zeros(1, np.int64))
    assert L.orbm_search_by_bow_many(0, None, None, None, F.ref(), fv.ref(), 0.75, 1, match, cnt) == 0
    assert L.orbm_search_for_triangulation_checked(None, None, None, None, None, None, 0, 1, abi.TRI_CHECK(0),
                                                    None, None) == PARAM
    assert L.orbx_extract_batch(None, 1, None, None, 64, 64, None, None, None, 0, None, None) == PARAM
