"""Prints the extraction plan (k_pyr_stream chunk rows, steps, LDS, fused pre-test) per image size."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam3_vio_fixes_amd import orb
ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
for w, h in [(752, 480), (512, 512), (640, 480), (320, 240), (1920, 1080)]:
    print(w, h, ex.plan_info(w, h))
