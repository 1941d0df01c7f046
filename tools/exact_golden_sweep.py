"""Every golden run of the real reference (tests/golden/manifest.json), replayed by the drop-in
executables in bit-exact mode on the GPU (development tool; the GPU box needs no reference).

For each (case, algorithm, P): `mpiexec -n P bin/multiplier_<alg> R C` with MVG_EXACT=1 (P > 1:
every rank on GPU 0, MVG_SAME_DEVICE=1), inputs from the reference's fixture files or the
synthetic spec (MVG_SYNTH=1, bit-identical to its %.4f text), y written by MVG_Y_OUT as "%.17g"
per line — compared byte for byte with the reference's own y dump of the same run. Block split
with more than two grid columns can differ in the last bit (the reference adds those partials in
message-arrival order, the exact mode in rank order). One JSON line per run.

    python tools/exact_golden_sweep.py [max_elements]
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402

MPIEXEC = "/opt/conda/bin/mpiexec"
GOLDEN = os.path.join(REPO, "tests", "golden")


def main():
    limit = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1 << 31
    manifest = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    with np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False) as z:
        golden = {k: z[k] for k in z.files}
    total = same = 0
    for case in manifest["cases"]:
        R, C = case["R"], case["C"]
        if R * C > limit:
            continue
        for alg, plist in case["runs"].items():
            for P in plist:
                with tempfile.TemporaryDirectory() as d:
                    os.makedirs(os.path.join(d, "data", "out"))
                    env = dict(os.environ, MVG_EXACT="1", MVG_ITERS="1", MVG_Y_OUT=os.path.join(d, "y.txt"))
                    if case["source"] == "fixture":
                        for f in ("matrix_4_8.txt", "vector_8.txt"):
                            shutil.copy(os.path.join(GOLDEN, f), os.path.join(d, "data", f))
                    else:
                        env["MVG_SYNTH"] = "1"
                    if P > 1:
                        env["MVG_SAME_DEVICE"] = "1"
                    r = subprocess.run([MPIEXEC, "-n", str(P), os.path.join(REPO, "bin", f"multiplier_{alg}"), str(R),
                                        str(C)], cwd=d, env=env, capture_output=True, text=True, timeout=600)
                    if r.returncode != 0:
                        print(json.dumps({"case": case["name"], "alg": alg, "P": P, "error": r.stderr[-500:]}))
                        sys.exit(1)
                    got = open(os.path.join(d, "y.txt")).read()
                want_y = golden[f"{case['name']}/{alg}/P{P}"]
                want = "".join("%.17g\n" % v for v in want_y)
                gc = mm.get_2_most_closest_multipliers(P)[1]
                y = np.array([float(v) for v in got.split()])
                line = {"case": case["name"], "R": R, "C": C, "alg": alg, "P": P,
                        "file_identical_to_reference": got == want,
                        "max_rel_vs_reference": float(np.max(np.abs(y - want_y) / np.maximum(np.abs(want_y), 1e-300)))}
                if alg == "blockwise" and gc > 2:
                    # bit identity with the rank-order combine is tests/test_gpu_exact.py's check
                    line["note"] = "reference adds these partials in message-arrival order"
                total += 1
                same += line["file_identical_to_reference"]
                print(json.dumps(line), flush=True)
    print(json.dumps({"runs": total, "files_identical": same}))


if __name__ == "__main__":
    main()
