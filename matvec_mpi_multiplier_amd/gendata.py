"""Input files for the reference's sweep, in its own format — the generator its repository lacks.

    python -m matvec_mpi_multiplier_amd.gendata R C [R C ...] [--dir ./data] [--test-sh]

The reference reads ./data/matrix_<R>_<C>.txt and ./data/vector_<C>.txt (matr_utils.c:9-18,
42-83): whitespace-separated "%lf" tokens, row-major, values written by numpy as "%.4f"
(README.md:26-37); the files are git-ignored there (.gitignore:3) and the script that made them
is not in the repository, so its test.sh cannot run from a fresh clone. This writes them from
the synthetic spec in include/matvec_gpu.h (seed 42 for A, 4242 for x: values k/10000, each
"%.4f" token parsing back to the same double), with the library's threaded writer, so the drop-in
executables (and the reference itself) can run the sweep; MVG_SYNTH=1 / =device skip the files
altogether. --test-sh writes the nine square sizes of test.sh:8 (600 ... 10200). Creates
<dir>/out/ as the executables expect.
"""
from __future__ import annotations

import argparse
import os

from . import multiplier as mm
from ._lib import SEED_A, SEED_X

TEST_SH_SIZES = (600, 1800, 3000, 4200, 5400, 6600, 7800, 9000, 10200)  # test.sh:8


def write_inputs(data_dir: str, R: int, C: int) -> tuple[str, str]:
    """matrix_R_C.txt and vector_C.txt under data_dir (the vector is shared by every R)."""
    os.makedirs(os.path.join(data_dir, "out"), exist_ok=True)
    mpath = os.path.join(data_dir, mm.build_matrix_filename(R, C))
    vpath = os.path.join(data_dir, mm.build_vector_filename(C))
    mm.write_matr_synth(mpath, R, C, SEED_A)
    if not os.path.exists(vpath):
        mm.write_matr_synth(vpath, 1, C, SEED_X)
    return mpath, vpath


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("sizes", nargs="*", type=int, help="R C pairs")
    ap.add_argument("--dir", default="./data")
    ap.add_argument("--test-sh", action="store_true", help="the nine square sizes of the reference's test.sh")
    args = ap.parse_args(argv)
    if len(args.sizes) % 2:
        ap.error("sizes come in R C pairs")
    pairs = list(zip(args.sizes[0::2], args.sizes[1::2]))
    if args.test_sh:
        pairs += [(n, n) for n in TEST_SH_SIZES]
    if not pairs:
        ap.error("nothing to write: give R C pairs or --test-sh")
    for R, C in pairs:
        m, v = write_inputs(args.dir, R, C)
        print(f"{m}  {v}")


if __name__ == "__main__":
    main()
