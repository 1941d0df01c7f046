"""BASELINE.json configs 2-5 at their own (R, C, P), through the drop-in executables, against the
real reference's own y.

tests/golden/config_slices.npz holds, per config and P, the reference's y (oracle/_ref under
mpiexec -n P, tests/golden/make_config_slices.py) on four bands of the config's rows — exactly
the y the reference gives those rows of the full problem, since a row's sum depends only on the
split of its columns (matr_utils.c:86-96, multiplier_colwise.c:107-124,
multiplier_blockwise.c:203-207,367). Here the executables run each config whole: P ranks under
`mpiexec -n P` (every rank on GPU 0, MVG_SAME_DEVICE=1 — the RCCL exchange runs over loopback
sockets; on a node with P GPUs the same command gives each rank its own GPU), or one process at
P = 1, inputs generated on the GPUs (MVG_SYNTH=device: config 4's 137 GB never exists on the
host), and their y file is compared on those rows:
  * default (tree-summed) mode: <= 1e-12 relative per element (north_star's bar);
  * MVG_EXACT=1: bit-identical — except the block split over more than two grid columns
    (config 4 at P = 8, a 2 x 4 grid), where the reference adds the partials in MPI_ANY_SOURCE
    arrival order (multiplier_blockwise.c:187,206): there y is bit-identical to the oracle's rank
    order and within 1e-12 of the reference's.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_DIR, REPO, max_rel

MPIEXEC = "/opt/conda/bin/mpiexec"
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no MPI launcher in this image")]

# (config, alg, R, C, P, exact): every config's P = 1 and P = 8 (the bench's scaling run's ends),
# the column and block splits also at 2 and 4, each mode at least once per config
RUNS = [
    ("cfg2", "rowwise", 16384, 16384, 1, False),
    ("cfg2", "rowwise", 16384, 16384, 8, True),
    ("cfg3", "colwise", 65536, 65536, 1, True),
    ("cfg3", "colwise", 65536, 65536, 2, False),
    ("cfg3", "colwise", 65536, 65536, 4, True),
    ("cfg3", "colwise", 65536, 65536, 8, False),
    ("cfg3", "colwise", 65536, 65536, 8, True),
    ("cfg4", "blockwise", 131072, 131072, 1, False),
    ("cfg4", "blockwise", 131072, 131072, 2, True),
    ("cfg4", "blockwise", 131072, 131072, 4, False),
    ("cfg4", "blockwise", 131072, 131072, 8, False),
    ("cfg4", "blockwise", 131072, 131072, 8, True),
    ("cfg5", "rowwise", 4194304, 512, 8, False),
    ("cfg5", "rowwise", 4194304, 512, 8, True),
]


@pytest.fixture(scope="module")
def slices():
    with np.load(os.path.join(GOLDEN_DIR, "config_slices.npz")) as z:
        return {k: z[k] for k in z.files}


def run_config(tmp_path, alg, R, C, P, exact):
    (tmp_path / "data" / "out").mkdir(parents=True)
    yout = tmp_path / "y.txt"
    env = dict(os.environ, MVG_SYNTH="device", MVG_ITERS="2", MVG_Y_OUT=str(yout),
               # the y file comes from the first multiply; no column-panel copies next to
               # config 4's 8 x 16 GiB shards on the one GPU
               MVG_NO_PANELS="1")
    if exact:
        env["MVG_EXACT"] = "1"
    exe = os.path.join(REPO, "bin", f"multiplier_{alg}")
    if P == 1:
        cmd = [exe, str(R), str(C)]
        env["MVG_NGPUS"] = "1"
    else:
        cmd = [MPIEXEC, "-n", str(P), exe, str(R), str(C)]
        env["MVG_SAME_DEVICE"] = "1"
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-3000:])
    assert "on the GPUs" in r.stdout
    y = np.fromfile(yout, dtype=np.float64, sep="\n")
    assert y.shape == (R,)
    csv = (tmp_path / "data" / "out" / f"{alg}.csv").read_text().splitlines()
    assert csv[1].startswith(f"{R}, {C}, {P}, "), csv
    return y


@pytest.mark.parametrize("cfg,alg,R,C,P,exact", RUNS)
def test_config_matches_reference_rows(tmp_path, slices, cfg, alg, R, C, P, exact):
    rows = slices[f"{cfg}/rows"]
    want = slices[f"{cfg}/{alg}/P{P}"]
    y = run_config(tmp_path, alg, R, C, P, exact)
    got = y[rows]
    assert np.all(np.isfinite(y)) and y.min() >= 0 and y.max() <= C * 0.9999 ** 2
    rel = max_rel(got, want)
    assert rel <= 1e-12, (cfg, alg, P, exact, rel)
    if not exact:
        return
    from oracle import oracle

    grid_cols = oracle.grid_shape(P)[1] if alg == "blockwise" else 1
    if grid_cols <= 2:
        assert np.array_equal(got, want), (cfg, alg, P, int(np.sum(got != want)))
    else:
        # arrival-order sums in the reference: the exact mode's rank order is the oracle's
        A = np.vstack([oracle.synth_block(int(b[0]), len(b), 0, C, C, 42)
                       for b in np.split(rows, np.flatnonzero(np.diff(rows) != 1) + 1)])
        x = oracle.synth(1, C, 4242)[0]
        assert np.array_equal(got, oracle.multiply(alg, A, x, P))
