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
