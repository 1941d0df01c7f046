"""The reference's benchmark sweep (test.sh:1-13) re-run with the drop-in executables.

    python tools/ref_sweep.py --out profiles/r01/ref_sweep_g1 [--gpus 1] [--iters 100]

For each algorithm, runs bin/multiplier_<alg> on the sizes the reference published
(data/out/{rowwise,colwise,blockwise}.csv: N x N, N = 600 ... 10200; and
data/out/asymmetric_*.csv: R x 60000, R = 120 ... 1200) with synthetic inputs (MVG_SYNTH=1; the
reference's text files were numpy-generated and are not in its repo) and the reference's own
timing semantics (100 iterations, each distributing A from the root's host memory, multiplying
and ending when the root holds y). Writes the executables' CSVs (same format as the reference's)
plus a JSON line per run with the device-resident time parsed from stdout.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SQUARE = [600, 1800, 3000, 4200, 5400, 6600, 7800, 9000, 10200]  # test.sh:8
ASYM_ROWS = [120, 240, 360, 480, 600, 720, 840, 960, 1080, 1200]  # asymmetric_*.csv
ASYM_COLS = 60000


def run(alg, R, C, gpus, iters, work):
    env = dict(os.environ, MVG_SYNTH="1", MVG_NGPUS=str(gpus), MVG_ITERS=str(iters))
    r = subprocess.run([os.path.join(REPO, "bin", f"multiplier_{alg}"), str(R), str(C)], cwd=work, env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"{alg} {R}x{C}: rc {r.returncode}\n{r.stdout[-1500:]}\n{r.stderr[-1500:]}")
    m = re.search(r"device-resident: ([0-9.]+) ms per multiply, ([0-9.]+) GB/s aggregate; GEMV kernel ([0-9.]+) ms",
                  r.stdout)
    e = re.search(r"end-to-end .*: mean ([0-9.]+) s", r.stdout)
    return {"alg": alg, "R": R, "C": C, "gpus": gpus, "iters": iters,
            "e2e_s": float(e.group(1)) if e else None,
            "device_ms": float(m.group(1)) if m else None,
            "device_GBps": float(m.group(2)) if m else None,
            "kernel_ms": float(m.group(3)) if m else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    summary = open(os.path.join(args.out, "runs.jsonl"), "w")
    for kind, shapes in (("square", [(n, n) for n in SQUARE]), ("asymmetric", [(r, ASYM_COLS) for r in ASYM_ROWS])):
        for alg in ("rowwise", "colwise", "blockwise"):
            with tempfile.TemporaryDirectory() as work:
                os.makedirs(os.path.join(work, "data", "out"))
                for R, C in shapes:
                    d = run(alg, R, C, args.gpus, args.iters, work)
                    d["set"] = kind
                    summary.write(json.dumps(d) + "\n")
                    summary.flush()
                    print(json.dumps(d), flush=True)
                name = f"{alg}.csv" if kind == "square" else f"asymmetric_{alg}.csv"
                shutil.copy(os.path.join(work, "data", "out", f"{alg}.csv"), os.path.join(args.out, name))
    summary.close()


if __name__ == "__main__":
    main()
