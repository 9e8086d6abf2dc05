#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: value, stage times, roofline.
usage: tools/bench_brief.py bench.json"""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
if "ms_per_step" not in d:                     # C3-C5 lines
    print(round(d["value"]), d.get("unit"), {k: d[k] for k in ("ms_per_query", "n_gpus", "near_frac", "parity")
                                            if k in d}, "roof", (d.get("roofline") or {}).get("frac"))
    sys.exit(0)
st = {k: round(v * 1e3, 1) for k, v in (d.get("stage_ms") or {}).items() if v}
r = d.get("roofline") or {}
print(round(d["value"]), "n_gpus", d.get("n_gpus"), "ms/step", round(d["ms_per_step"], 4), st,
      "roof", r.get("kernel"), r.get("frac") and round(r["frac"], 4),
      "parity", d.get("parity", {}).get("frames_mismatched"), d.get("parity", {}).get("pairs_mismatched"))
