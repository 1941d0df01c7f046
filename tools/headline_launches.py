"""The headline's timed launches in a rocprofv3 kernel trace of bench.py (development tool).

    python tools/headline_launches.py <rocprofv3 output dir> [--steps 20] [--bench line.json] [--out f.json]

bench.py's headline runs one GEMV instantiation back to back: the settle, the W warm-up steps and
the K timed steps, and then the exact section starts with a different kernel. So the K timed
launches are the last K launches of the first long run of one kernel name and grid before another
kernel appears. Writes their per-launch durations (us), their mean and the span from the first
start to the last end, beside the line's own span-timed `roofline.kernel_ms` when --bench names
the line.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def launches(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                grid = 1
                for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"):
                    grid *= int(r.get(k, 1) or 1)
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid))
    rows.sort()
    return rows


def headline(rows, steps, min_run=100):
    """The last `steps` launches of the first run of >= `min_run` launches of one (kernel, grid)
    that no other kernel interrupts (RCCL's own kernels, the exchange, aside)."""
    run, key = [], None
    for r in rows:
        if r[2:] == key:
            run.append(r)
        elif "nccl" in r[2].lower():
            continue
        else:
            if len(run) >= min_run:
                break
            run, key = [r], r[2:]
    return run[-steps:] if len(run) >= min_run else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--bench")
    ap.add_argument("--out")
    args = ap.parse_args()
    sel = headline(launches(args.dir), args.steps)
    if not sel:
        raise SystemExit("no run of one kernel long enough to be the headline")
    us = [round((e - s) / 1e3, 3) for s, e, _, _ in sel]
    out = {"kernel": sel[0][2], "grid_threads": sel[0][3],
           "note": f"the headline's K = {len(sel)} timed launches: the last {len(sel)} launches of the first long "
                   "run of one kernel (settle, warm-up, timed steps) before the exact section's first kernel",
           "launch_us": us, "mean_us": round(statistics.mean(us), 3),
           "first_start_to_last_end_us": round((sel[-1][1] - sel[0][0]) / 1e3, 3)}
    if args.bench:
        line = json.loads([ln for ln in open(args.bench) if ln.startswith("{")][-1])
        out["line_kernel_us"] = round(line["roofline"]["kernel_ms"] * 1e3, 3)
        out["line_value"] = line["value"]
    text = json.dumps(out, indent=1)
    if args.out:
        open(args.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
