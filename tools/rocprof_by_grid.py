"""Per-launch-shape summary of a rocprofv3 kernel trace (development tool).

    python tools/rocprof_by_grid.py <rocprofv3 output dir> [--out file.csv]

rocprofv3 --stats averages every launch of a kernel name together. bench.py launches the same
GEMV instantiation for several workloads (config 2, then configs 3-5 in its `configs` section),
so this groups the kernel-trace rows by (kernel name, grid size) instead: one row per workload,
with launch count and mean / min / max duration in microseconds.
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    args = ap.parse_args()
    groups = defaultdict(list)
    for path in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                grid = tuple(int(r.get(k, 0) or 0) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
                wg = int(r.get("Workgroup_Size_X", 0) or 0)
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                groups[(r["Kernel_Name"], grid[0] * grid[1] * grid[2], wg)].append(dur)
    rows = []
    for (name, grid, wg), d in sorted(groups.items(), key=lambda t: -sum(t[1])):
        rows.append({"kernel": name, "grid_threads": grid, "workgroup": wg, "workgroups": grid // max(wg, 1),
                     "launches": len(d), "mean_us": round(statistics.mean(d), 3),
                     "median_us": round(statistics.median(d), 3), "min_us": round(min(d), 3),
                     "max_us": round(max(d), 3), "total_ms": round(sum(d) / 1e3, 3)})
    out = open(args.out, "w", newline="") if args.out else None
    w = csv.DictWriter(out or __import__("sys").stdout, fieldnames=list(rows[0]) if rows else ["kernel"])
    w.writeheader()
    w.writerows(rows)
    if out:
        out.close()


if __name__ == "__main__":
    main()
