"""Summarise rocprofv3 PMC passes for the GEMV kernel into profiles/<round>/pmc_<tag>.json.

    python tools/pmc_traffic.py --out profiles/r01/pmc_rowwise_16384.json --alg rowwise --R 16384 --C 16384 \
        gpurun_out/pmc_fetch gpurun_out/pmc_write [gpurun_out/pmc_l2 ...]

Each directory holds one `rocprofv3 --pmc ... --output-format csv` pass (counters collected in
separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass). HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly
half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B stores and uncalibrated for the GEMV's 8-B y stores (which are 8 B per row,
negligible next to the A stream).
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def read_counters(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            rows += list(csv.DictReader(f))
    per = defaultdict(dict)  # dispatch -> {counter: value}
    names = {}
    for r in rows:
        kname = r.get("Kernel_Name", "")
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        cname = r.get("Counter_Name")
        val = float(r.get("Counter_Value", "nan"))
        per[disp][cname] = per[disp].get(cname, 0.0) + val
        names[disp] = kname
    return per, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--alg", required=True)
    ap.add_argument("--R", type=int, required=True)
    ap.add_argument("--C", type=int, required=True)
    ap.add_argument("--kernel", default="mvg::gemv_")
    ap.add_argument("--bytes-per-launch", type=int, default=None)
    args = ap.parse_args()
    counters = defaultdict(list)
    for d in args.dirs:
        per, names = read_counters(d)
        for disp, cs in per.items():
            if args.kernel in names[disp]:
                for c, v in cs.items():
                    counters[c].append(v)
    med = {c: statistics.median(v) for c, v in counters.items()}
    algo = args.bytes_per_launch or 8 * (args.R * args.C + args.C + args.R)
    out = {"alg": args.alg, "R": args.R, "C": args.C, "kernel": args.kernel,
           "launches": {c: len(v) for c, v in counters.items()}, "median_counters": med,
           "algorithmic_bytes_per_launch": algo}
    if "FETCH_SIZE" in med:
        fetch = 2.0 * med["FETCH_SIZE"] * 1024.0  # gfx950: FETCH_SIZE = half of a wide stream
        write = med.get("WRITE_SIZE", 0.0) * 1024.0
        out["hbm_read_bytes_per_launch"] = fetch
        out["hbm_write_bytes_per_launch"] = write
        out["hbm_bytes_per_launch"] = int(fetch + write)
        out["traffic_over_algorithmic"] = (fetch + write) / algo
        out["correction"] = "FETCH_SIZE x 1024 x 2 (gfx950 wide-stream half count) + WRITE_SIZE x 1024"
    for derived in ("VALUBusy", "VALUUtilization", "MemUnitStalled", "TA_BUSY_avr"):
        if derived in med:
            out[derived] = med[derived]
    if "GRBM_GUI_ACTIVE" in med:
        out["note_clock"] = "effective clock ~ GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md)"
    if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
        tot = med["TCC_HIT_sum"] + med["TCC_MISS_sum"]
        out["l2_hit_rate"] = med["TCC_HIT_sum"] / tot if tot else None
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
