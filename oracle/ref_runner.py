"""Runs the REAL reference (oracle/_ref/multiplier_<alg>, built by oracle/build_ref.sh from the
reference's own sources) under MPICH's mpiexec — TEST INFRASTRUCTURE ONLY.

Used by bench.py's cpu_baseline leg (kind "reference") to time the reference's CPU path on the
GPU box's host cores, and available to tests. The reference reads ./data/matrix_R_C.txt and
./data/vector_C.txt relative to its working directory (matr_utils.c:10,16,45,68), times its own
100-iteration loop (multiplier_rowwise.c:135-151, colwise.c:218-233, blockwise.c:361-378) and
appends "R, C, P, time" to ./data/out/<alg>.csv (rowwise.c:160-169); oracle/ref_dump.h makes rank
0 dump y to $ORACLE_Y. Inputs are the synthetic values in the reference's own "%.4f" text form
(include/matvec_gpu.h spec), so y is directly comparable with the GPU's y on the same rows.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BIN = os.path.join(HERE, "_ref")
MPIEXEC = os.environ.get("MVG_MPIEXEC", "/opt/conda/bin/mpiexec")


def available(alg: str) -> bool:
    return os.access(os.path.join(REF_BIN, f"multiplier_{alg}"), os.X_OK) and os.access(MPIEXEC, os.X_OK)


def write_inputs(data_dir: str, R: int, C: int, seed_a: int = 42, seed_x: int = 4242) -> None:
    """The synthetic A and x as the reference's text files (values k/10000, "%.4f")."""
    from matvec_mpi_multiplier_amd._lib import check, lib

    check(lib.mvg_write_matr_synth(os.path.join(data_dir, f"matrix_{R}_{C}.txt").encode(), R, C, seed_a),
          "mvg_write_matr_synth")
    check(lib.mvg_write_matr_synth(os.path.join(data_dir, f"vector_{C}.txt").encode(), 1, C, seed_x),
          "mvg_write_matr_synth")


_TOKENS = None


def write_synth_rows(path: str, rows: np.ndarray, C: int, seed: int) -> None:
    """Rows `rows` (global indices, any order) of the synthetic R x C matrix, stacked, as the
    reference's text (one "%.4f" token per value, README.md:32). Every value is k/10000 with
    k < 10000, so its text is "0.dddd"; one 7-byte token per value from a table, written
    band by band (a few hundred MB per second)."""
    from oracle import oracle

    global _TOKENS
    if _TOKENS is None:
        _TOKENS = np.frombuffer(b"".join(b"0.%04d " % k for k in range(10000)), dtype=np.uint8).reshape(10000, 7)
    rows = np.asarray(rows, dtype=np.int64)
    # contiguous runs of global rows, each generated at once
    cuts = np.flatnonzero(np.diff(rows) != 1) + 1
    step = max(1, (64 << 20) // max(1, 8 * C))
    with open(path, "wb") as f:
        for run_rows in np.split(rows, cuts):
            for b in range(0, len(run_rows), step):
                r0, nr = int(run_rows[b]), int(min(step, len(run_rows) - b))
                k = np.rint(oracle.synth_block(r0, nr, 0, C, C, seed) * 10000.0).astype(np.int32)
                assert k.min() >= 0 and k.max() < 10000
                txt = _TOKENS[k].reshape(nr, 7 * C)
                txt[:, -1] = ord("\n")
                f.write(txt.tobytes())


def run_tracked(cmd, timeout, track=None, **kw) -> subprocess.CompletedProcess:
    """subprocess.run in a session of its own (mpiexec and its ranks form one process group):
    the group is killed when the time limit passes, and while it runs the Popen sits in `track`
    (a set), so a caller that is being terminated can end the group too (bench.py's watcher)."""
    import signal

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True, **kw)
    if track is not None:
        track.add(p)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.communicate()
        raise
    finally:
        if track is not None:
            track.discard(p)
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def run(alg: str, R: int, C: int, P: int, timeout: float = 300.0, workdir: str | None = None,
        cpus: list[int] | None = None, rows: np.ndarray | None = None, track: set | None = None) -> dict:
    """mpiexec -n P multiplier_<alg> R C in a scratch directory. Returns {"seconds": mean time
    per iteration as the reference printed it, "y": rank 0's y, "wall_s": whole run incl. text
    loading}. With `cpus`, mpiexec and every rank it starts (MPICH's hydra does not bind by
    default, so ranks inherit the launcher's affinity) run confined to those CPUs. With `rows`
    (global row indices of the synthetic R x C matrix), the reference runs on just those rows,
    stacked into a len(rows) x C matrix: a row's sum depends only on the split of its columns
    (matr_utils.c:86-96, multiplier_colwise.c:107-122, multiplier_blockwise.c:367), so y is the
    reference's own y for those rows of the full problem at the same P (whenever the column
    split is the same: row split, column split, and block split on grids that divide both).
    `track`: a set that holds the run's Popen while it runs (run_tracked). Raises RuntimeError
    on any failure."""
    if not available(alg):
        raise RuntimeError(f"reference executable or {MPIEXEC} missing")
    own = workdir is None
    work = workdir or tempfile.mkdtemp(prefix="mvg_ref_")
    try:
        data = os.path.join(work, "data")
        os.makedirs(os.path.join(data, "out"), exist_ok=True)
        if rows is None:
            write_inputs(data, R, C)
        else:
            R = len(rows)
            write_synth_rows(os.path.join(data, f"matrix_{R}_{C}.txt"), rows, C, 42)
            write_synth_rows(os.path.join(data, f"vector_{C}.txt"), np.zeros(1, dtype=np.int64), C, 4242)
        csv = os.path.join(data, "out", f"{alg}.csv")
        if os.path.exists(csv):
            os.remove(csv)
        ypath = os.path.join(work, "y.txt")
        env = dict(os.environ, ORACLE_Y=ypath)
        cmd = [MPIEXEC, "-n", str(P), os.path.join(REF_BIN, f"multiplier_{alg}"), str(R), str(C)]
        t0 = time.perf_counter()
        pin = (lambda: os.sched_setaffinity(0, cpus)) if cpus else None
        r = run_tracked(cmd, timeout, track, cwd=work, env=env, preexec_fn=pin)
        wall = time.perf_counter() - t0
        if r.returncode != 0 or not os.path.exists(csv) or not os.path.exists(ypath):
            raise RuntimeError(f"reference {alg} P={P} failed (rc {r.returncode}): {r.stdout[-400:]} {r.stderr[-400:]}")
        last = [ln for ln in open(csv).read().splitlines() if ln.strip()][-1]
        seconds = float(last.split(",")[3])
        y = np.loadtxt(ypath, dtype=np.float64, ndmin=1)
        return {"seconds": seconds, "y": y, "wall_s": wall}
    finally:
        if own:
            shutil.rmtree(work, ignore_errors=True)
