"""Compare tools/ref_sweep.py output with the reference's published CSVs (run where
/root/reference exists). Writes a markdown table next to the sweep output."""
import csv
import json
import os
import sys

REF = "/root/reference/data/out"


def load_ref(name):
    out = {}
    with open(os.path.join(REF, name)) as f:
        for row in csv.DictReader(f):
            row = {k.strip(): v.strip() for k, v in row.items()}
            out.setdefault((int(row["n_rows"]), int(row["n_cols"])), {})[int(row["n_processes"])] = float(row["time"])
    return out


def main(sweep_dir):
    runs = [json.loads(l) for l in open(os.path.join(sweep_dir, "runs.jsonl"))]
    lines = ["# Reference sweep (test.sh sizes) — drop-in executables on MI355X vs the published CPU CSVs", "",
             "Reference: `data/out/*.csv` (i5-10400F, MPI, mean of 100 iterations, distribution from the root "
             "included). Here: `bin/multiplier_<alg>` on 1 MI355X, same timing semantics (end-to-end: root's "
             "host A -> GPU -> y on the root), and the device-resident time (A already in HBM).", "",
             "| alg | shape | ref P=1 | ref best (P) | MI355X end-to-end | speed-up vs best | device-resident | speed-up vs best |",
             "|---|---|---|---|---|---|---|---|"]
    for r in runs:
        name = f"{r['alg']}.csv" if r["set"] == "square" else f"asymmetric_{r['alg']}.csv"
        ref = load_ref(name).get((r["R"], r["C"]), {})
        if not ref:
            continue
        best_p = min(ref, key=ref.get)
        best = ref[best_p]
        lines.append(f"| {r['alg']} | {r['R']}x{r['C']} | {ref.get(1, float('nan'))*1e3:.1f} ms | "
                     f"{best*1e3:.1f} ms ({best_p}) | {r['e2e_s']*1e3:.2f} ms | {best/r['e2e_s']:.0f}x | "
                     f"{r['device_ms']*1e3:.1f} us | {best/(r['device_ms']*1e-3):.0f}x |")
    out = os.path.join(sweep_dir, "comparison.md")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
