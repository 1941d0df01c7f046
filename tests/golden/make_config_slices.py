"""Reference y for BASELINE.json configs 2-5 at their own (R, C, P) — TEST INFRASTRUCTURE.

The reference cannot run the configs whole here (2-137 GB of text, int overflows in its MPI
counts at configs 3-4, a crash of MPICH's 2 GiB MPI_Scatter at config 2). It does not need to:
a row's sum depends only on how its columns are split (matr_utils.c:86-96 for the row split,
multiplier_colwise.c:107-124 for the column split, multiplier_blockwise.c:367 + 203-207 for the
block split), never on the other rows. So the reference's own executables (oracle/_ref, built
from its sources by oracle/build_ref.sh) run with `mpiexec -n P` on a matrix made of a few bands
of the config's rows — at the top, a third and two thirds down, and at the bottom — with the
config's full width C and the config's P, give the reference's y for exactly those rows of the
full problem. (MPI_Reduce of the column split picks its algorithm by message size, n * 8 >
2048 bytes and n >= pof2; the bands hold >= 512 rows, so the slice takes the same algorithm as
the full 65536 rows, and at P = 1, 2, 4, 8 every algorithm sums in the same order anyway.)

Writes tests/golden/config_slices.npz: "<cfg>/rows" = the global row indices, "<cfg>/<alg>/P<p>"
= the reference's y on them; and config_slices.json (shapes, bands, seeds, the reference's own
mean time per iteration on this container's CPUs, for information).

Usage: python tests/golden/make_config_slices.py [--only cfg3,...]   (needs /root/reference and
the image's MPICH).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

# name, alg, R, C, P list (BASELINE.json configs[1..4]); P = 1 is the one-GPU run of the same
# config, the others the GPU counts the bench's scaling run uses
CONFIGS = [
    ("cfg2", "rowwise", 16384, 16384, [1, 8]),
    ("cfg3", "colwise", 65536, 65536, [1, 2, 4, 8]),
    ("cfg4", "blockwise", 131072, 131072, [1, 2, 4, 8]),
    ("cfg5", "rowwise", 4194304, 512, [1, 8]),
]


def band_rows(R: int, C: int) -> np.ndarray:
    """Four bands of `band` rows: top, a third down, two thirds down, bottom (band a multiple of
    8 so the stacked slice splits over every P and grid used here)."""
    band = max(128, (1 << 20) // C // 8 * 8)
    starts = [0, R // 3 // 8 * 8, 2 * R // 3 // 8 * 8, R - band]
    return np.concatenate([np.arange(s, s + band, dtype=np.int64) for s in starts])


def main() -> None:
    from oracle import ref_runner

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    only = [n for n in ap.parse_args().only.split(",") if n]
    subprocess.run([os.path.join(REPO, "oracle", "build_ref.sh")], check=True)
    npz = os.path.join(HERE, "config_slices.npz")
    out: dict[str, np.ndarray] = {}
    meta = {"generator": "tests/golden/make_config_slices.py", "reference": "oracle/_ref (MPICH 3.3.2, gcc -O0)",
            "seed_a": 42, "seed_x": 4242, "configs": []}
    if only and os.path.exists(npz):
        with np.load(npz) as old:
            out = {k: old[k] for k in old.files if k.split("/")[0] not in only}
        with open(os.path.join(HERE, "config_slices.json")) as f:
            meta["configs"] = [c for c in json.load(f)["configs"] if c["name"] not in only]
    for name, alg, R, C, plist in CONFIGS:
        if only and name not in only:
            continue
        rows = band_rows(R, C)
        out[f"{name}/rows"] = rows
        entry = {"name": name, "alg": alg, "R": R, "C": C, "rows": int(len(rows)),
                 "band_starts": [int(rows[0]), *(int(r) for r in rows[1:][np.diff(rows) != 1])], "runs": {}}
        for p in plist:
            t0 = time.perf_counter()
            r = ref_runner.run(alg, R, C, p, timeout=3600, rows=rows)
            y = r["y"]
            assert y.shape == rows.shape, (name, p, y.shape)
            out[f"{name}/{alg}/P{p}"] = y
            entry["runs"][f"P{p}"] = {"ref_seconds_per_iter": r["seconds"], "wall_s": round(time.perf_counter() - t0, 1)}
            print(f"{name} {alg} P={p}: {len(rows)} rows x {C}, y[0]={y[0]!r}, "
                  f"{r['seconds']:.4f} s/iter, {time.perf_counter() - t0:.0f} s", flush=True)
        meta["configs"].append(entry)
    meta["configs"].sort(key=lambda c: c["name"])
    np.savez_compressed(npz, **out)
    with open(os.path.join(HERE, "config_slices.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote {len(out)} arrays to {npz}")


if __name__ == "__main__":
    main()
