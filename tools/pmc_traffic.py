"""Summarise rocprofv3 PMC passes (tools/pmc_passes.sh) into one JSON per GEMV kernel family.

    python tools/pmc_traffic.py --outdir profiles/r04 --M 16384 --K 16384 [--pieces 1] \
        gpurun_out/<run>/pmc/<variant>

Every directory below the given ones holds one `rocprofv3 --pmc ... --output-format csv` pass
(counters collected in separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
Dispatches are grouped by kernel family (the template name: gemv_rowblock, gemv_vec,
gemv_seq_hop, gemv_seq_hop_panel, ...), each family's counters reduced to the median over its
dispatches, and written to OUTDIR/pmc_<family>_<M>x<K>.json. `--pieces n`: the library splits
one call into n equal launches (config 5's short rows go out in 1 GiB launches), so one dispatch
carries 1/n of the shape's algorithmic bytes.

Derived fields (MI355X_MICROARCH.md §HBM and §rocprofv3; rocprofv3 sums a counter over its
dimensions in the CSV, so GRBM_GUI_ACTIVE is the sum over the 8 XCDs):
  hbm_bytes_per_launch  FETCH_SIZE x 1024 x 2 (gfx950 reports half of a wide stream) + WRITE_SIZE x 1024
  valu_busy             SQ_ACTIVE_INST_VALU (quad-cycles, summed over SIMDs) / 256 CUs / (GRBM_GUI_ACTIVE / 8):
                        the fraction of SIMD cycles issuing vector ALU work (rocprofv3's VALUBusy / 100)
  l2_hit                TCC_HIT / (TCC_HIT + TCC_MISS)
  ea_read_latency_cyc   TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ: mean cycles an L2 read miss is in flight
  ea_reads_in_flight    TCC_EA0_RDREQ_LEVEL / (GRBM_GUI_ACTIVE / 8): mean memory-side reads in flight
  dram_read_frac        TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ: reads the L2 sends to the HBM controllers.
                        gfx950 exposes no Infinity-Cache (MALL) hit counter to rocprofv3 (no MALL_*
                        block in `rocprofv3 -L`); its hits are inside these requests.
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict

CUS, XCDS = 256, 8


def family(kernel_name: str) -> str:
    """The template name; the multi-wave (evenly placed) hop forms, gemv_seq_hop<L, W, U, B, NW>
    with NW > 1, are a family of their own (gemv_seq_hop_n<NW>), as bench.kernel_family names
    them."""
    m = re.search(r"mvg::(\w+)(?:<([^>]*)>)?", kernel_name)
    if not m:
        return kernel_name.split("(")[0]
    fam, targs = m.group(1), [a.strip() for a in (m.group(2) or "").split(",") if a.strip()]
    if fam == "gemv_seq_hop" and len(targs) >= 5 and targs[4].isdigit() and int(targs[4]) > 1:
        return f"{fam}_n{int(targs[4])}"
    return fam


def read_dirs(dirs):
    """{family: {counter: [value per dispatch]}} and the full template name seen per family."""
    vals = defaultdict(lambda: defaultdict(list))
    names = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(dict)
            kn = {}
            with open(path) as f:
                for r in csv.DictReader(f):
                    disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                    c = r["Counter_Name"]
                    per[disp][c] = per[disp].get(c, 0.0) + float(r["Counter_Value"])
                    kn[disp] = r.get("Kernel_Name", "")
            for disp, cs in per.items():
                fam = family(kn[disp])
                if not fam.startswith("gemv"):
                    continue  # the synthetic fill, the panel relayout
                names[fam] = kn[disp].split("(")[0].replace("void ", "")
                for c, v in cs.items():
                    vals[fam][c].append(v)
    return vals, names


def derive(med: dict, algo: int) -> dict:
    out = {}
    grbm = med.get("GRBM_GUI_ACTIVE")
    if "FETCH_SIZE" in med:
        fetch = 2.0 * med["FETCH_SIZE"] * 1024.0
        write = med.get("WRITE_SIZE", 0.0) * 1024.0
        out.update(hbm_read_bytes_per_launch=fetch, hbm_write_bytes_per_launch=write,
                   hbm_bytes_per_launch=int(fetch + write), traffic_over_algorithmic=(fetch + write) / algo,
                   correction="FETCH_SIZE x 1024 x 2 (gfx950 wide-stream half count) + WRITE_SIZE x 1024")
    if "SQ_ACTIVE_INST_VALU" in med and grbm:
        out["valu_busy"] = med["SQ_ACTIVE_INST_VALU"] / CUS / (grbm / XCDS)
    if "SQ_INSTS_VALU" in med and "SQ_WAVES" in med and med["SQ_WAVES"]:
        out["valu_insts_per_wave"] = med["SQ_INSTS_VALU"] / med["SQ_WAVES"]
    if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
        tot = med["TCC_HIT_sum"] + med["TCC_MISS_sum"]
        out["l2_hit"] = med["TCC_HIT_sum"] / tot if tot else None
    rd = med.get("TCC_EA0_RDREQ_sum")
    if rd:
        if "TCC_EA0_RDREQ_LEVEL_sum" in med:
            out["ea_read_latency_cyc"] = med["TCC_EA0_RDREQ_LEVEL_sum"] / rd
            if grbm:
                out["ea_reads_in_flight"] = med["TCC_EA0_RDREQ_LEVEL_sum"] / (grbm / XCDS)
        if "TCC_EA0_RDREQ_DRAM_sum" in med:
            out["dram_read_frac"] = med["TCC_EA0_RDREQ_DRAM_sum"] / rd
    if "TCP_UTCL1_REQUEST_sum" in med and med["TCP_UTCL1_REQUEST_sum"]:
        out["utcl1_miss_rate"] = med.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0) / med["TCP_UTCL1_REQUEST_sum"]
    if grbm:
        out["grbm_cycles_per_xcd"] = grbm / XCDS
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--outdir", required=True)
    ap.add_argument("--M", type=int, required=True, help="rows of the shape the probe multiplied")
    ap.add_argument("--K", type=int, required=True)
    ap.add_argument("--pieces", type=int, default=1, help="equal launches the library splits one call into")
    ap.add_argument("--only", default=None, help="comma-separated kernel families to write")
    args = ap.parse_args()
    vals, names = read_dirs(args.dirs)
    algo = 8 * (args.M * args.K + args.K + args.M) // args.pieces
    os.makedirs(args.outdir, exist_ok=True)
    for fam, cs in sorted(vals.items()):
        if args.only and fam not in args.only.split(","):
            continue
        med = {c: statistics.median(v) for c, v in cs.items()}
        out = {"kernel_family": fam, "kernel": names[fam], "M": args.M, "K": args.K, "pieces": args.pieces,
               "dispatches": {c: len(v) for c, v in cs.items()}, "median_counters": med,
               "algorithmic_bytes_per_launch": algo, **derive(med, algo),
               "sources": [os.path.relpath(d) for d in args.dirs]}
        path = os.path.join(args.outdir, f"pmc_{fam}_{args.M}x{args.K}.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(path, json.dumps({k: out[k] for k in out if k in (
            "traffic_over_algorithmic", "valu_busy", "l2_hit", "ea_read_latency_cyc", "ea_reads_in_flight",
            "dram_read_frac", "utcl1_miss_rate")}))


if __name__ == "__main__":
    main()
