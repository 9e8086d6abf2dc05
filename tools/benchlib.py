"""Shared measurement helpers of bench.py's workloads:
per-stage HIP-event profiles of an extractor handle and the roofline of the
FAST pass (every pyramid pixel read once) against the HBM peak."""
from __future__ import annotations

import numpy as np

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
STAGES = ["pyramid", "fast_cells", "quadtree", "describe", "assemble"]


def level_sizes(ex, w: int, h: int) -> list[int]:
    """Pixels of each pyramid level (ComputePyramid sizes, ORBextractor.cc:1174-1175)."""
    return [int(np.rint(np.float32(w) * np.float32(s))) * int(np.rint(np.float32(h) * np.float32(s)))
            for s in ex.GetInverseScaleFactors()]


def profile_on(exs):
    from orb_slam3_vio_fixes_amd import capi
    for ex in exs:
        capi.check(capi.lib().orbx_set_profiling(ex._h, 1), "orbx_set_profiling")


def profile_read(exs):
    """Per-launch average stage times (ms) over every recorded call of the
    handles, and the number of calls; profiling is switched off."""
    from orb_slam3_vio_fixes_amd import capi
    tot = np.zeros(len(STAGES), np.float64)
    calls = 0
    for ex in exs:
        st = np.zeros(len(STAGES), np.float32)
        c = capi.lib().orbx_get_profile(ex._h, st.ctypes.data, len(STAGES))
        capi.lib().orbx_set_profiling(ex._h, 0)
        tot += st
        calls += max(0, c)
    return {k: float(v) / max(1, calls) for k, v in zip(STAGES, tot)}, calls


def fast_roofline(ex, w: int, h: int, stage_ms: dict, frames_per_launch: float) -> dict:
    """roofline object of the FAST pass (k_fast_cells): algorithmic bytes =
    sum of the level sizes x frames per launch, over its HIP-event time."""
    px = sum(level_sizes(ex, w, h))
    ms = float(stage_ms.get("fast_cells") or 0)
    ach = px * frames_per_launch / (ms * 1e-3) / 1e9 if ms > 0 else None
    return {"kernel": "k_fast_cells", "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS if ach else None, "traffic": None,
            "bytes_per_launch": px * frames_per_launch, "ms_per_launch": ms, "frames_per_launch": frames_per_launch}
