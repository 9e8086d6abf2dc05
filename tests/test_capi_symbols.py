"""The product library loads without a GPU and exports every function the C
header declares (no compute calls)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "orb_mi355x.h"


def declared():
    txt = re.sub(r"/\*.*?\*/", " ", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(orb[xmvsk]_[a-z0-9_]+)\s*\(", txt)))


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


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from orb_slam3_vio_fixes_amd import orb
    with pytest.raises(RuntimeError):
        orb.ORBextractor(1000, 1.2, 8, 20, 7)
