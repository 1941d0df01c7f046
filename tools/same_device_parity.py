"""Multi-rank parity on a one-GPU machine (development tool): the executables launched as
`mpiexec -n P bin/multiplier_<alg> R C` with every rank on GPU 0 (MVG_SAME_DEVICE=1: RCCL over
loopback sockets), y compared with the real reference's golden y for the same P."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    with np.load(os.path.join(REPO, "tests", "golden", "golden.npz")) as z:
        golden = {k: z[k] for k in z.files}
    cases = [("sq_480", 480, 480, a, p) for a in ("rowwise", "colwise", "blockwise") for p in (2, 3, 4)]
    cases += [("wide_120x6000", 120, 6000, a, 4) for a in ("rowwise", "colwise", "blockwise")]
    ok = True
    for name, R, C, alg, p in cases:
        with tempfile.TemporaryDirectory() as work:
            os.makedirs(os.path.join(work, "data", "out"))
            yout = os.path.join(work, "y.txt")
            env = dict(os.environ, MVG_SYNTH="1", MVG_SAME_DEVICE="1", MVG_ITERS="3", MVG_Y_OUT=yout)
            for dist in ("shared", "send"):
                if dist == "send":
                    env["MVG_DIST"] = "send"
                r = subprocess.run(["/opt/conda/bin/mpiexec", "-n", str(p), os.path.join(REPO, "bin", f"multiplier_{alg}"),
                                    str(R), str(C)], cwd=work, env=env, capture_output=True, text=True, timeout=240)
                if r.returncode != 0:
                    print(json.dumps({"case": name, "alg": alg, "P": p, "dist": dist, "rc": r.returncode,
                                      "err": r.stderr[-800:]}), flush=True)
                    ok = False
                    continue
                y = np.loadtxt(yout)
                want = golden[f"{name}/{alg}/P{p}"]
                rel = float(np.max(np.abs(y - want) / np.abs(want)))
                line = [l for l in r.stdout.splitlines() if l.startswith("launch:")]
                print(json.dumps({"case": name, "alg": alg, "P": p, "dist": dist, "max_rel_vs_reference": rel,
                                  "launch": line[0] if line else None}), flush=True)
                ok &= rel <= 1e-12
    print("ALL_OK" if ok else "FAILED", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
