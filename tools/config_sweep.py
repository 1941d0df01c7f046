"""Run bench.py over the BASELINE.json configs on the GPUs of this box (the reference's
test.sh sweep, re-aimed at the MI355X configs) and collect one JSON line per run.

    python tools/config_sweep.py --out profiles/r01/configs_g1.jsonl [--gpus 1] [--only cfg3,cfg5]

Config 1 (the 4x8 fixture, P = 2 on the CPU) is a parity case (tests/), not a bench line.
At G = 1 every config runs on one GPU whole: config 3 is a 32 GiB strip set, config 4 the
137 GB matrix as a 1 x 1 grid, config 5 the 16 GiB tall-skinny matrix.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    "cfg2": ["--alg", "rowwise", "--rows", "16384", "--cols", "16384"],
    "cfg3": ["--alg", "colwise", "--rows", "65536", "--cols", "65536"],
    "cfg4": ["--alg", "blockwise", "--rows", "131072", "--cols", "131072", "--e2e-iters", "1", "--steps", "20"],
    "cfg5": ["--alg", "rowwise", "--rows", "4194304", "--cols", "512"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--only", default="")
    ap.add_argument("--timeout", type=int, default=600)
    args, extra = ap.parse_known_args()
    only = [c for c in args.only.split(",") if c]
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "a") as f:
        for name, cargs in CONFIGS.items():
            if only and name not in only:
                continue
            cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(args.gpus)] + cargs + extra
            if args.gpus > 1:
                cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                       "--master-addr", "127.0.0.1", "--master-port", "29512"] + cmd[1:]
            t0 = time.time()
            print(f"== {name}: {' '.join(cmd[-12:])}", flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
            line = next((l for l in r.stdout.splitlines() if l.startswith("{")), None)
            if r.returncode != 0 or line is None:
                print(r.stdout[-2000:], r.stderr[-2000:], flush=True)
                raise SystemExit(f"{name} failed (rc {r.returncode})")
            d = json.loads(line)
            d["sweep_config"] = name
            d["wall_s"] = round(time.time() - t0, 1)
            f.write(json.dumps(d) + "\n")
            f.flush()
            e2e = d.get("end_to_end") or {}
            sh = e2e.get("shared") if isinstance(e2e.get("shared"), dict) else {}
            print(f"   value {d['value']} GB/s, kernel {d['roofline']['achieved']} GB/s "
                  f"({d['roofline']['frac']:.3f} of peak), step {d['ms_per_step']} ms, "
                  f"e2e {sh.get('mean_s')}, cpu {(d.get('cpu_baseline') or {}).get('value')}", flush=True)


if __name__ == "__main__":
    main()
