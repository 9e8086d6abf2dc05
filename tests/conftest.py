import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under `pytest -m gpu`)")
    config.addinivalue_line("markers", "slow: long CPU test")


def have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real device; fail loudly (no CPU fallback)."""
    if not have_gpu():
        pytest.fail("gpu test selected but no GPU is visible")
    from orb_slam3_vio_fixes_amd import capi
    return capi.lib()


@pytest.fixture
def debug_option():
    """Sets orb_debug_set_option values (alternative kernel forms, a test hook of
    include/orb_mi355x.h) for one test and restores them afterwards."""
    from orb_slam3_vio_fixes_amd import capi
    L = capi.lib()
    saved = {}

    def set_(option, value):
        saved.setdefault(option, L.orb_debug_get_option(option))
        capi.check(L.orb_debug_set_option(option, value), "orb_debug_set_option")
    yield set_
    for option, value in saved.items():
        L.orb_debug_set_option(option, value)


@pytest.fixture
def proj_form(debug_option):
    """Projection-search form by name: fused (one launch: brute-force top-K +
    last-block fixpoint resolve, the default), serial (top-K + serial resolve),
    single (single-wave search), spec (top-K + speculative resolve),
    fused_nogrid (the fused form scanning the whole frame per window)."""
    from orb_slam3_vio_fixes_amd import capi

    def set_(name):
        debug_option(capi.ORB_OPT_PROJ_FORM, {"fused": 0, "serial": 1, "single": 2, "spec": 3, "fused_nogrid": 4, "fused_split": 5}[name])
    return set_


@pytest.fixture
def sfi_form(debug_option):
    """Host SearchForInitialization form by name: fused (one launch: brute-force
    top-K + last-block fixpoint resolve, the default) or grid (grid order +
    top-K + serial resolve) or fused_nogrid (fused, scanning all of F2)."""
    from orb_slam3_vio_fixes_amd import capi

    def set_(name):
        debug_option(capi.ORB_OPT_SFI_FORM, {"fused": 0, "grid": 1, "fused_nogrid": 2, "fused_split": 3}[name])
    return set_
