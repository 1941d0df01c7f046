"""Speed-up and efficiency from the timing CSVs (the reference's offline metrics, README.md:47-50).

    python -m matvec_mpi_multiplier_amd.stats data/out/rowwise.csv [more.csv ...]

Reads the CSV the executables append to (`n_rows, n_cols, n_processes, time`, rowwise.c:86,168)
— also the reference's published, space-less header — and prints, per (n_rows, n_cols), the
speed-up S = T_serial / T_parallel and efficiency E = S / p with T_serial the p = 1 time
(the plots of the missing stats_visualization.ipynb, as a table).
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def read_times(path: str) -> dict[tuple[int, int], dict[int, float]]:
    """{(n_rows, n_cols): {p: mean seconds}}; a repeated (shape, p) keeps the last row."""
    out: dict[tuple[int, int], dict[int, float]] = defaultdict(dict)
    with open(path, newline="") as f:
        for row in csv.DictReader(f, skipinitialspace=True):
            row = {k.strip(): v.strip() for k, v in row.items() if k is not None}
            out[(int(row["n_rows"]), int(row["n_cols"]))][int(row["n_processes"])] = float(row["time"])
    return dict(out)


def speedup_efficiency(times: dict[int, float]) -> list[dict]:
    """README.md:47-50: S = T_serial / T_parallel, E = S / p (T_serial = the p = 1 time)."""
    if 1 not in times:
        raise ValueError("no p = 1 time to take as T_serial")
    t1 = times[1]
    return [{"p": p, "time": t, "speedup": t1 / t, "efficiency": t1 / t / p} for p, t in sorted(times.items())]


def table(path: str) -> str:
    lines = [f"# {path}", "| n_rows | n_cols | p | time (s) | speed-up | efficiency |", "|---|---|---|---|---|---|"]
    for (r, c), times in sorted(read_times(path).items()):
        if 1 not in times:
            continue
        for d in speedup_efficiency(times):
            lines.append(f"| {r} | {c} | {d['p']} | {d['time']:.6f} | {d['speedup']:.3f} | {d['efficiency']:.3f} |")
    return "\n".join(lines)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(table(p))
