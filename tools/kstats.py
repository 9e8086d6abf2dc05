#!/usr/bin/env python3
"""Per-kernel statistics of a rocprofv3 kernel trace, split by launch grid:
the bench's batch-256 launches and the host-API leg's one-image launches of
the same kernel otherwise share one average in the --stats summary.
--last N averages only the last N launches of each (kernel, grid): bench.py's
profiled pass (one step in flight, after the timed steps) is the last
--profile-steps launches of every 256-frame extraction kernel, the launches
whose HIP-event times the bench line's roofline reports.
usage: tools/kstats.py run_kernel_trace.csv [--csv out.csv] [--last N]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    d = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        grid = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}'
        d[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if last:
        d = {k: v[-last:] for k, v in d.items()}
    out = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    w = None
    if "--csv" in sys.argv:
        w = csv.writer(open(sys.argv[sys.argv.index("--csv") + 1], "w"))
        w.writerow(["kernel", "grid", "calls", "avg_us", "min_us", "max_us", "total_us"])
    for (name, grid), v in out:
        row = [name, grid, len(v), sum(v) / len(v) / 1e3, min(v) / 1e3, max(v) / 1e3, sum(v) / 1e3]
        if w:
            w.writerow(row)
        print(f"{name[:60]:60s} {grid:22s} n={len(v):5d} avg={row[3]:9.2f}us min={row[4]:9.2f} max={row[5]:9.2f}")


if __name__ == "__main__":
    main()
