"""Per-kernel summary of the PMC passes written by tools/pmc_profile.sh.

usage: python tools/pmc_summary.py <outdir> [--csv out.csv]

Per kernel (averaged over its dispatches): duration, waves, VALU / LDS / SALU
instructions per wave, the wait / issue-stall / active fractions of wave
cycles, the LDS bank-conflict ratio, FETCH_SIZE (x2: gfx950 reports half the
bytes of wide streaming reads, MI355X_MICROARCH.md HBM section) and WRITE_SIZE
in MB per dispatch, and the VALU issue fraction: VALU wave-instructions per
second over the chip's 2 per CU per cycle (4 SIMD-32 units, wave64 over 2
cycles) at the effective clock GRBM_GUI_ACTIVE / 8 XCDs / duration.
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

CUS = 256


def load(outdir):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
    dur = defaultdict(dict)                          # kernel -> dispatch -> ns
    for f in glob.glob(os.path.join(outdir, "p*", "*counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                d = (f, row["Dispatch_Id"])
                per[(k, d)][row["Counter_Name"]] += float(row["Counter_Value"])
                dur[k][d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        for (k, d), cs in per.items():
            for c, v in cs.items():
                vals[k][c].append(v)
    return vals, dur


def summarize(outdir):
    vals, dur = load(outdir)
    rows = []
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sum(dur[k].values()) / max(1, len(dur[k])) / 1e3
        waves = avg.get("SQ_WAVES", 0.0)
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        r = {"kernel": k, "dispatches": len(dur[k]), "us": us, "waves": waves}
        if waves:
            for c, n in (("SQ_INSTS_VALU", "valu_per_wave"), ("SQ_INSTS_LDS", "lds_per_wave"),
                         ("SQ_INSTS_SALU", "salu_per_wave")):
                if c in avg:
                    r[n] = avg[c] / waves
        if wc:
            for c, n in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_ACTIVE_INST_ANY", "active")):
                if c in avg:
                    r[n] = avg[c] / wc
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
        if waves:
            for c, n in (("SQ_INSTS_VMEM_RD", "vmem_rd_per_wave"), ("SQ_INSTS_VMEM_WR", "vmem_wr_per_wave"),
                         ("SQ_INSTS_SMEM", "smem_per_wave")):
                if c in avg:
                    r[n] = avg[c] / waves
        if wc:
            for c, n in (("SQ_WAIT_INST_LDS", "lds_wait"), ("SQ_ACTIVE_INST_LDS", "lds_active"),
                         ("SQ_ACTIVE_INST_VMEM", "vmem_active")):
                if c in avg:
                    r[n] = avg[c] / wc
        if avg.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_ADDR_CONFLICT" in avg:
            r["lds_addr_conflict"] = avg["SQ_LDS_ADDR_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        if gui_ta := avg.get("GRBM_GUI_ACTIVE"):
            if "TA_TA_BUSY" in avg:
                r["ta_busy"] = avg["TA_TA_BUSY"] / (gui_ta / 8 * CUS)
            if "TA_ADDR_STALLED_BY_TC_CYCLES" in avg:
                r["ta_addr_stall_tc"] = avg["TA_ADDR_STALLED_BY_TC_CYCLES"] / (gui_ta / 8 * CUS)
        if "FETCH_SIZE" in avg:
            r["fetch_MB_x2"] = 2 * avg["FETCH_SIZE"] / 1024          # FETCH_SIZE is in KB
        if "WRITE_SIZE" in avg:
            r["write_MB"] = avg["WRITE_SIZE"] / 1024
        gui = avg.get("GRBM_GUI_ACTIVE")
        if gui and us > 0:
            clk_ghz = gui / 8 / (us * 1e3)
            r["clock_GHz"] = clk_ghz
            if "SQ_INSTS_VALU" in avg:
                peak = 2 * CUS * clk_ghz * 1e9             # wave-instructions / s
                r["valu_issue_frac"] = avg["SQ_INSTS_VALU"] / (us * 1e-6) / peak
        rows.append(r)
    rows.sort(key=lambda r: -r["us"] * r["dispatches"])
    return rows


def main():
    outdir = sys.argv[1]
    rows = summarize(outdir)
    keys = ["kernel", "dispatches", "us", "waves", "valu_per_wave", "lds_per_wave", "salu_per_wave", "wait",
            "issue_stall", "active", "lds_conflict", "fetch_MB_x2", "write_MB", "clock_GHz", "valu_issue_frac",
            "vmem_rd_per_wave", "vmem_wr_per_wave", "smem_per_wave", "lds_wait", "lds_active", "vmem_active",
            "lds_addr_conflict", "ta_busy", "ta_addr_stall_tc"]
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=keys, extrasaction="ignore")
            w.writeheader()
            for r in rows:
                w.writerow({k: (f"{r[k]:.4g}" if isinstance(r.get(k), float) else r.get(k, "")) for k in keys})
    for r in rows:
        print(" ".join(f"{k}={r[k]:.4g}" if isinstance(r.get(k), float) else f"{k}={r.get(k)}"
                       for k in keys if k in r))


if __name__ == "__main__":
    main()
