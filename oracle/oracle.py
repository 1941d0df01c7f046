"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
as the checker or as the CPU baseline; the product (matvec_mpi_multiplier_amd) never does.
See oracle/cpu_ref.c for what each function restates (reference file:line).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MVG_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # `make asan` build
ALGS = {"rowwise": 0, "colwise": 1, "blockwise": 2}


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    dp = C.c_void_p
    lib.ref_multiply_std_rowwise.argtypes = [dp, dp, C.c_int64, C.c_int64, dp]
    lib.ref_multiply_std_rowwise.restype = None
    lib.ref_grid_shape.argtypes = [C.c_int64, C.POINTER(C.c_int)]
    lib.ref_grid_shape.restype = None
    lib.ref_multiply.argtypes = [C.c_int, dp, dp, C.c_int64, C.c_int64, C.c_int, dp]
    lib.ref_multiply.restype = C.c_int
    lib.ref_synth_value.argtypes = [C.c_uint64, C.c_uint64]
    lib.ref_synth_value.restype = C.c_double
    lib.ref_synth_fill.argtypes = [dp, C.c_int64, C.c_int64, C.c_uint64]
    lib.ref_synth_fill.restype = None
    lib.ref_synth_block.argtypes = [dp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_uint64]
    lib.ref_synth_block.restype = None
    lib.ref_time_multiply.argtypes = [C.c_int, dp, dp, C.c_int64, C.c_int64, C.c_int, C.c_int, dp]
    lib.ref_time_multiply.restype = C.c_double
    lib.ref_mpich_reduce.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int64]
    lib.ref_mpich_reduce.restype = None
    return lib


lib = _load()


def _c(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def multiply_std_rowwise(A: np.ndarray, x: np.ndarray) -> np.ndarray:
    """src/matr_utils.c:86-96 — sequential left-to-right fp64 sum per row."""
    A, x = _c(A), _c(x)
    R, Cn = A.shape
    y = np.empty(R, dtype=np.float64)
    lib.ref_multiply_std_rowwise(A.ctypes.data, x.ctypes.data, R, Cn, y.ctypes.data)
    return y


def multiply(alg: str, A: np.ndarray, x: np.ndarray, P: int) -> np.ndarray:
    """The reference's distributed result for `alg` at P ranks (rank-order reductions)."""
    A, x = _c(A), _c(x)
    R, Cn = A.shape
    y = np.empty(max(R, 1), dtype=np.float64)
    rc = lib.ref_multiply(ALGS[alg], A.ctypes.data, x.ctypes.data, R, Cn, P, y.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle: {alg} {R}x{Cn} does not split over P={P}")
    return y[:R]


def mpich_reduce(parts: list[np.ndarray]) -> np.ndarray:
    """MPI_Reduce(SUM, root 0) of the ranks' partial y in the order the reference's MPICH 3.3.2
    sums them (multiplier_colwise.c:124; binomial tree, or reduce-scatter + gather above 2 KiB,
    oracle/cpu_ref.c ref_mpich_reduce)."""
    bufs = [_c(p).copy() for p in parts]
    n = bufs[0].shape[0]
    ptrs = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    lib.ref_mpich_reduce(ptrs, len(bufs), n)
    return bufs[0]


def grid_shape(p: int) -> tuple[int, int]:
    """src/utils.c:26-37."""
    d = (C.c_int * 2)(0, 0)
    lib.ref_grid_shape(p, d)
    return d[0], d[1]


def synth(R: int, Cn: int, seed: int) -> np.ndarray:
    out = np.empty((R, Cn), dtype=np.float64)
    if R * Cn:
        lib.ref_synth_fill(out.ctypes.data, R, Cn, seed)
    return out


def synth_block(r0: int, nr: int, c0: int, nc: int, Cn: int, seed: int) -> np.ndarray:
    """Rows [r0, r0+nr) x cols [c0, c0+nc) of the synthetic R x Cn matrix."""
    out = np.empty((nr, nc), dtype=np.float64)
    if nr * nc:
        lib.ref_synth_block(out.ctypes.data, r0, nr, c0, nc, Cn, seed)
    return out


def synth_value(seed: int, idx: int) -> float:
    return lib.ref_synth_value(seed, idx)


def time_multiply(alg: str, A: np.ndarray, x: np.ndarray, P: int, iters: int) -> tuple[float, np.ndarray]:
    """Reference timing semantics with P threads as ranks: mean over iterations of the
    per-iteration max over ranks, distribution included. Returns (seconds, y)."""
    A, x = _c(A), _c(x)
    R, Cn = A.shape
    y = np.empty(max(R, 1), dtype=np.float64)
    t = lib.ref_time_multiply(ALGS[alg], A.ctypes.data, x.ctypes.data, R, Cn, P, iters, y.ctypes.data)
    if t < 0:
        raise ValueError("oracle timing: bad shape for P")
    return t, y[:R]
