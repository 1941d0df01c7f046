"""Generate tests/golden/golden.npz from the REAL reference (TEST INFRASTRUCTURE).

Runs the reference's own three executables, compiled from /root/reference/src by
oracle/build_ref.sh into oracle/_ref/ (with MPICH, as in the reference's test.sh), on:
  * the reference's own fixture data/matrix_4_8.txt x data/vector_8.txt (copied here as data),
  * synthetic inputs written in the reference's text format ("%.4f", README.md:32) from the
    generator spec in include/matvec_gpu.h (seeds 42 for A, 4242 for x),
at several process counts, and stores rank 0's y (dumped by oracle/ref_dump.h) keyed
"<case>/<alg>/P<p>". Only the y vectors (and the two tiny fixture files) are committed;
synthetic matrices are regenerated bit-exactly from (seed, R, C).

Usage: python tests/golden/make_golden.py [--only NAME,...]   (needs /root/reference and
/opt/conda MPICH). --only regenerates just those cases and keeps the others' vectors.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402

MPIEXEC = "/opt/conda/bin/mpiexec"
REF_BIN = os.path.join(REPO, "oracle", "_ref")

ALL = ("rowwise", "colwise", "blockwise")
# name, R, C, source, {alg: [P, ...]}
CASES = [
    ("fixture_4x8", 4, 8, "fixture", {"rowwise": [1, 2, 4], "colwise": [1, 2, 4, 8], "blockwise": [1, 2, 4, 8]}),
    ("odd_5x7", 5, 7, "synth", {"rowwise": [1, 5], "colwise": [1, 7], "blockwise": [1, 7]}),
    ("sq_480", 480, 480, "synth", {a: [1, 2, 3, 4, 6, 8] for a in ALL}),
    # colwise P = 5, 6 at R = 120: MPICH's binomial MPI_Reduce (120 * 8 bytes <= 2048)
    ("wide_120x6000", 120, 6000, "synth", {"rowwise": [1, 2, 4, 8], "colwise": [1, 2, 4, 5, 6, 8],
                                           "blockwise": [1, 2, 4, 8]}),
    # colwise at non-power-of-two P with R = 720 (> 2048 bytes): MPICH's reduce-scatter + gather
    # MPI_Reduce, whose sum order differs from the binomial tree's at P = 5, 9, 10 (3, 6, 12 agree)
    ("sq_720", 720, 720, "synth", {"colwise": [1, 2, 3, 5, 6, 8, 9, 10, 12]}),
    # column split is left out for R > C: the reference corrupts its heap there
    # (multiplier_colwise.c:115 sizes `columns` by n_cols, SURVEY §4 bug 2).
    ("tall_960x96", 960, 96, "synth", {"rowwise": [1, 2, 4, 8], "blockwise": [1, 2, 3, 4, 8]}),
    ("sq_4200", 4200, 4200, "synth", {a: [1, 2, 4, 8] for a in ALL}),
    # config 2's 16384-row matrix at half its width (1 GiB, 0.95 GB of text): the full 16384^2
    # segfaults in this build (2^31 bytes through one MPI_Scatter; the reference's own counts
    # stay below 2^31, so most likely a limit of MPICH 3.3.2)
    ("big_16384x8192", 16384, 8192, "synth", {"rowwise": [4, 8], "blockwise": [4, 8]}),
    ("big_8192x16384", 8192, 16384, "synth", {"colwise": [4, 8]}),  # R <= C for the column split
]


def write_inputs(data_dir: str, name: str, R: int, C: int, source: str) -> None:
    if source == "fixture":
        for f in ("matrix_4_8.txt", "vector_8.txt"):
            shutil.copy(os.path.join(HERE, f), os.path.join(data_dir, f))
        return
    x = oracle.synth(1, C, 4242)[0]
    if R * C > (1 << 24):
        # large: the library's "%.4f" writer (numpy's savetxt would take minutes); the values
        # are the same k/10000 the oracle generates, and every test compares against y anyway
        from matvec_mpi_multiplier_amd import multiplier as mm

        mm.write_matr_synth(os.path.join(data_dir, f"matrix_{R}_{C}.txt"), R, C, 42)
    else:
        A = oracle.synth(R, C, 42)
        np.savetxt(os.path.join(data_dir, f"matrix_{R}_{C}.txt"), A, fmt="%.4f")
    np.savetxt(os.path.join(data_dir, f"vector_{C}.txt"), x, fmt="%.4f")


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="comma-separated case names to (re)generate")
    only = [n for n in ap.parse_args().only.split(",") if n]
    subprocess.run([os.path.join(REPO, "oracle", "build_ref.sh")], check=True)
    out: dict[str, np.ndarray] = {}
    manifest = {"generator": "tests/golden/make_golden.py", "reference": "oracle/_ref (MPICH 3.3.2, gcc -O0)",
                "seed_a": 42, "seed_x": 4242, "cases": []}
    if only:  # keep every other case's vectors and manifest entry
        with np.load(os.path.join(HERE, "golden.npz")) as old:
            out = {k: old[k] for k in old.files if k.split("/")[0] not in only}
        with open(os.path.join(HERE, "manifest.json")) as f:
            kept = {c["name"]: c for c in json.load(f)["cases"] if c["name"] not in only}
    with tempfile.TemporaryDirectory() as work:
        data = os.path.join(work, "data")
        os.makedirs(os.path.join(data, "out"))
        for name, R, C, source, plan in CASES:
            if only and name not in only:
                if name in kept:
                    manifest["cases"].append(kept[name])
                continue
            write_inputs(data, name, R, C, source)
            manifest["cases"].append({"name": name, "R": R, "C": C, "source": source, "runs": plan})
            for alg, plist in plan.items():
                for p in plist:
                    ypath = os.path.join(work, "y.txt")
                    if os.path.exists(ypath):
                        os.remove(ypath)
                    env = dict(os.environ, ORACLE_Y=ypath)
                    cmd = [MPIEXEC, "-n", str(p), os.path.join(REF_BIN, f"multiplier_{alg}"), str(R), str(C)]
                    r = subprocess.run(cmd, cwd=work, env=env, capture_output=True, text=True, timeout=1800)
                    if r.returncode != 0 or not os.path.exists(ypath):
                        raise RuntimeError(f"{name} {alg} P={p} failed: {r.stdout[-500:]} {r.stderr[-500:]}")
                    y = np.loadtxt(ypath, dtype=np.float64, ndmin=1)
                    assert y.shape == (R,), (name, alg, p, y.shape)
                    out[f"{name}/{alg}/P{p}"] = y
                    print(f"{name:16s} {alg:9s} P={p}: y[0]={y[0]!r}", flush=True)
            for f in os.listdir(data):
                if f.endswith(".txt"):
                    os.remove(os.path.join(data, f))
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(out)} golden vectors")


if __name__ == "__main__":
    main()
