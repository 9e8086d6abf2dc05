"""Builds the HIP library in-tree: orb_slam3_vio_fixes_amd/liborb_mi355x.so.

hipcc for gfx950 only; -ffp-contract=off because the reference's float
semantics are reproduced with explicit fmaf()/fma().
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "liborb_mi355x.so"
SOURCES = ["extractor.hip", "matcher.hip", "stereo.hip", "kfdb.hip", "vocab.cpp"]
DEPS = SOURCES + ["common.h", "orb_math.h", "plan.h", "brief_pattern.inc", "host_gather.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wno-unused-result"]
# (MFMA accumulators live in VGPRs, the compiler's own choice: round 2's C5
# failures in that form came from an inline-asm key reading an accumulator
# the hazard recognizer could not see, fixed in round 3)


def stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / d for d in DEPS] + [PKG.parent / "include" / "orb_mi355x.h"]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not stale():
        return LIB
    cmd = [HIPCC, *FLAGS, *[str(CSRC / s) for s in SOURCES], "-o", str(LIB)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
