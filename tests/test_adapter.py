"""The drop-in ORBextractor adapter (adapters/orbslam3/ORBextractor.cc)
compiles against the reference's own, unmodified include/ORBextractor.h
(include/ORBextractor.h:43-109) and this repository's C ABI.  OpenCV is absent
from the image, so tests/native/cv_decl/ declares the subset of its API that
the header and the adapter use (syntax check only: nothing is linked or run).
Skipped where the reference tree is not present (the GPU box)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF_INC = Path("/root/reference/include")


@pytest.mark.skipif(not (REF_INC / "ORBextractor.h").exists(), reason="reference tree not present")
@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_extractor_adapter_compiles_against_reference_header():
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
           "-I", str(ROOT / "tests" / "native" / "cv_decl"), "-I", str(REF_INC), "-I", str(ROOT / "include"),
           str(ROOT / "adapters" / "orbslam3" / "ORBextractor.cc")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_adapter_uses_only_declared_abi():
    """Every orbx_/orbm_ function the adapters call is declared in include/orb_mi355x.h."""
    import re
    header = (ROOT / "include" / "orb_mi355x.h").read_text()
    declared = set(re.findall(r"\b((?:orbx|orbm|orbs|orbv|orbk)_[a-z0-9_]+)\s*\(", header))
    for src in (ROOT / "adapters" / "orbslam3").glob("*.cc"):
        used = set(re.findall(r"\b((?:orbx|orbm|orbs|orbv|orbk)_[a-z0-9_]+)\s*\(", src.read_text()))
        assert used <= declared, (src.name, used - declared)
