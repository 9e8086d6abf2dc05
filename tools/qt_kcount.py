#!/usr/bin/env python3
"""FAST keypoints per level (the quadtree's K) on the bench's synthetic frames (single-frame path)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam3_vio_fixes_amd import orb, synth

ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
frames = synth.sequence(752, 480, 16, config=2)
ks = []
for i in range(16):
    ex(np.ascontiguousarray(frames[i]))
    ks.append([len(x) for x in ex.debug_stage(0)])
ks = np.array(ks)
print("K per level (mean / max over 16 frames):")
print(" ".join(f"{m:.0f}/{x}" for m, x in zip(ks.mean(0), ks.max(0))))
