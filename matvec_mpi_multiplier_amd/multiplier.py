"""Host-side mirror of the reference's interface, over libmatvec_gpu.so.

Reference names are kept so a user of the MPI lab code finds the same operations:

  multiply_std_rowwise(A, x)          src/matr_utils.c:86-96   (runs the HIP GEMV on cuda:0;
                                      exact=True: bit-identical to the reference's sum)
  get_2_most_closest_multipliers(p)   src/utils.c:26-37
  load_matr / load_vec                src/matr_utils.c:42-83   (same file names, "%lf" tokens)
  build_matrix_filename / build_vector_filename   src/matr_utils.c:9-18
  Multiplier(alg, R, C, comm)         the three drivers' distribute -> multiply -> collect
                                      (src/multiplier_{rowwise,colwise,blockwise}.c)

Every compute call goes to the HIP library; nothing here computes a product on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import ALG_BY_NAME, ALG_NAMES, SEED_A, SEED_X, IndivisibleError, Shard, XStep, check, lib, runtime_info  # noqa: F401


def _alg_id(alg) -> int:
    if isinstance(alg, str):
        return ALG_BY_NAME[alg]
    return int(alg)


# ------------------------------------------------------------------ planner (no GPU)
def get_2_most_closest_multipliers(p: int) -> tuple[int, int]:
    """(grid rows, grid cols) = (largest d <= sqrt(p) dividing p, p / d) — src/utils.c:26-37."""
    r, c = C.c_int(), C.c_int()
    check(lib.mvg_grid_shape(p, C.byref(r), C.byref(c)), "mvg_grid_shape")
    return r.value, c.value


def plan_shard(alg, R: int, Cn: int, nranks: int, rank: int) -> Shard:
    s = Shard()
    check(lib.mvg_plan_shard(_alg_id(alg), R, Cn, nranks, rank, C.byref(s)), "mvg_plan_shard")
    return s


def plan_exchange(alg, R: int, Cn: int, nranks: int, rank: int, force_collect: bool = False) -> list[XStep]:
    steps = (XStep * _lib.MAX_XSTEPS)()
    n = C.c_int()
    check(lib.mvg_plan_exchange(_alg_id(alg), R, Cn, nranks, rank, int(force_collect), steps,
                                _lib.MAX_XSTEPS, C.byref(n)), "mvg_plan_exchange")
    return [steps[i] for i in range(n.value)]


# ------------------------------------------------------------------ text I/O
def trace_exchange(alg, R: int, Cn: int, ndev: int, exact: bool = False) -> list[dict]:
    """The calls one process driving `ndev` devices issues for the exchange (communicator splits,
    then one multiply's collectives; mvg_debug_trace_exchange), as dicts in issue order."""
    cap = 16 * ndev + 16
    calls = (_lib.XCall * cap)()
    n = C.c_int()
    check(lib.mvg_debug_trace_exchange(_alg_id(alg), R, Cn, ndev, int(exact), calls, cap, C.byref(n)),
          "mvg_debug_trace_exchange")
    return [calls[i].as_dict() for i in range(n.value)]


def build_matrix_filename(R: int, Cn: int) -> str:
    buf = C.create_string_buffer(128)
    check(lib.mvg_matrix_filename(R, Cn, buf, 128), "mvg_matrix_filename")
    return buf.value.decode()


def build_vector_filename(n: int) -> str:
    buf = C.create_string_buffer(128)
    check(lib.mvg_vector_filename(n, buf, 128), "mvg_vector_filename")
    return buf.value.decode()


def load_matr(R: int, Cn: int, data_dir: str = "./data") -> np.ndarray:
    A = np.empty((R, Cn), dtype=np.float64)
    check(lib.mvg_load_matr(data_dir.encode(), R, Cn, A.ctypes.data), "load_matr")
    return A


def load_vec(n: int, data_dir: str = "./data") -> np.ndarray:
    x = np.empty(n, dtype=np.float64)
    check(lib.mvg_load_vec(data_dir.encode(), n, x.ctypes.data), "load_vec")
    return x


def write_vec(path: str, v: np.ndarray) -> None:
    v = np.ascontiguousarray(v, dtype=np.float64)
    check(lib.mvg_write_vec(path.encode(), v.ctypes.data, v.size), "write_vec")


def write_matr_bin(path: str, A: np.ndarray) -> None:
    """The binary cache load_matr prefers over the text when present (see matvec_gpu.h)."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    check(lib.mvg_write_matr_bin(path.encode(), A.ctypes.data, A.shape[0], A.shape[1]), "write_matr_bin")


def write_matr_synth(path: str, R: int, Cn: int, seed: int) -> None:
    check(lib.mvg_write_matr_synth(path.encode(), R, Cn, seed), "write_matr_synth")


def synth_host(R: int, Cn: int, seed: int) -> np.ndarray:
    """The synthetic input (include/matvec_gpu.h spec) on the host."""
    A = np.empty((R, Cn), dtype=np.float64)
    check(lib.mvg_synth_fill_host(A.ctypes.data, Cn, R, Cn, 0, 0, Cn, seed), "mvg_synth_fill_host")
    return A


# ------------------------------------------------------------------ device buffers
class DeviceBuffer:
    """hipMalloc'd fp64 buffer owned by the library's allocator (current device)."""

    def __init__(self, n: int):
        self.n = int(n)
        p = C.c_void_p()
        check(lib.mvg_malloc(C.byref(p), max(self.n, 1) * 8), "mvg_malloc")
        self.ptr = p.value

    def upload(self, a: np.ndarray, stream=None) -> "DeviceBuffer":
        a = np.ascontiguousarray(a, dtype=np.float64)
        if a.size > self.n:
            raise ValueError(f"upload of {a.size} doubles into a buffer of {self.n}")
        check(lib.mvg_memcpy_h2d(self.ptr, a.ctypes.data, a.size * 8, stream), "h2d")
        check(lib.mvg_stream_sync(stream), "sync")
        return self

    def download(self, n: int | None = None, stream=None) -> np.ndarray:
        n = self.n if n is None else n
        out = np.empty(n, dtype=np.float64)
        check(lib.mvg_memcpy_d2h(out.ctypes.data, self.ptr, n * 8, stream), "d2h")
        check(lib.mvg_stream_sync(stream), "sync")
        return out

    def free(self) -> None:
        if self.ptr:
            lib.mvg_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def gemv(d_A: int, lda: int, d_x: int, d_y: int, m: int, k: int, stream=None, variant: int = 0,
         exact: bool = False) -> None:
    """y = A x on device pointers (the raw kernel: mvg_gemv, or mvg_gemv_exact)."""
    if exact:
        check(lib.mvg_gemv_exact_variant(d_A, lda, d_x, d_y, m, k, variant, stream), "mvg_gemv_exact")
    else:
        check(lib.mvg_gemv_variant(d_A, lda, d_x, d_y, m, k, variant, stream), "mvg_gemv")


def multiply_multi(A: np.ndarray, X: np.ndarray) -> np.ndarray:
    """Y = A X for a k x nv block of vectors in one pass over A (mvg_gemv_multi); returns m x nv."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    R, Cn = A.shape
    nv = X.shape[1]
    Xc = np.ascontiguousarray(X.T)  # column-major: vector v contiguous
    dA, dX, dY = DeviceBuffer(R * Cn).upload(A), DeviceBuffer(Cn * nv).upload(Xc), DeviceBuffer(R * nv)
    try:
        check(lib.mvg_gemv_multi(dA.ptr, Cn, dX.ptr, Cn, dY.ptr, R, R, Cn, nv, None), "mvg_gemv_multi")
        check(lib.mvg_stream_sync(None), "sync")
        return dY.download(R * nv).reshape(nv, R).T.copy()
    finally:
        for b in (dA, dX, dY):
            b.free()


def multiply_std_rowwise(A: np.ndarray, x: np.ndarray, variant: int = 0, exact: bool = False) -> np.ndarray:
    """src/matr_utils.c:86-96 on the GPU: copies A, x to the current device, runs the HIP
    GEMV, returns y. Matches the reference's sequential sum to <= 1e-12 relative; with
    exact=True (mvg_gemv_exact) bit for bit."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    R, Cn = A.shape
    if x.shape != (Cn,):
        raise ValueError(f"x has shape {x.shape}, A has {Cn} columns")
    dA, dx, dy = DeviceBuffer(R * Cn).upload(A), DeviceBuffer(Cn).upload(x), DeviceBuffer(R)
    try:
        gemv(dA.ptr, Cn, dx.ptr, dy.ptr, R, Cn, None, variant, exact)
        check(lib.mvg_stream_sync(None), "sync")
        return dy.download(R)
    finally:
        for b in (dA, dx, dy):
            b.free()


# ------------------------------------------------------------------ communicators
class Comm:
    """RCCL communicator(s) for the devices this process drives."""

    def __init__(self, handle: int):
        self.handle = handle

    @classmethod
    def init_all(cls, devices: list[int]) -> "Comm":
        """Single process, all `devices` (ncclCommInitAll) — the executables' model."""
        arr = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(lib.mvg_comm_init_all(C.byref(h), len(devices), arr), "mvg_comm_init_all")
        return cls(h.value)

    @classmethod
    def init_rank(cls, uid: bytes, nranks: int, rank: int, device: int) -> "Comm":
        h = C.c_void_p()
        check(lib.mvg_comm_init_rank(C.byref(h), uid, nranks, rank, device), "mvg_comm_init_rank")
        return cls(h.value)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(_lib.UNIQUE_ID_BYTES)
        check(lib.mvg_comm_unique_id(buf), "mvg_comm_unique_id")
        return buf.raw

    @classmethod
    def from_process_group(cls, device: int) -> "Comm":
        """One process per GPU under torch.distributed(.run): rank 0 makes the RCCL unique id,
        the default process group carries it to every rank (any backend, gloo included)."""
        uid = broadcast_unique_id(cls.unique_id)
        import torch.distributed as dist

        return cls.init_rank(uid, dist.get_world_size(), dist.get_rank(), device)

    @property
    def size(self) -> int:
        n = C.c_int()
        check(lib.mvg_comm_size(self.handle, C.byref(n)), "mvg_comm_size")
        return n.value

    def destroy(self) -> None:
        if self.handle:
            lib.mvg_comm_destroy(self.handle)
            self.handle = None


def broadcast_unique_id(make_id) -> bytes:
    """Rank 0 calls make_id(); every rank returns those 128 bytes (torch.distributed
    broadcast over the default group, CPU tensor for gloo, device tensor for nccl)."""
    import torch
    import torch.distributed as dist

    dev = "cpu"
    if dist.get_backend() == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    t = torch.zeros(_lib.UNIQUE_ID_BYTES, dtype=torch.uint8, device=dev)
    if dist.get_rank() == 0:
        uid = make_id()
        assert len(uid) == _lib.UNIQUE_ID_BYTES
        t.copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
    dist.broadcast(t, src=0)
    return bytes(t.cpu().numpy().tobytes())


# ------------------------------------------------------------------ the distributed multiplier
@dataclass
class KernelTiming:
    avg_ms: float
    launches: int


class Multiplier:
    """One distributed multiplier (alg, R x C) over a Comm. The drivers' loop body
    (distribute_data -> local product -> gather/reduce, e.g. multiplier_rowwise.c:139-141)
    maps to distribute() -> multiply() -> collect(). exact=True: y bit-identical to the
    reference's (mvg_engine_set_exact); None leaves the MVG_EXACT environment default."""

    def __init__(self, alg, R: int, Cn: int, comm: Comm, exact: bool | None = None):
        self.alg = _alg_id(alg)
        self.R, self.C = int(R), int(Cn)
        self.comm = comm
        h = C.c_void_p()
        check(lib.mvg_engine_create(C.byref(h), self.alg, self.R, self.C, comm.handle), "mvg_engine_create")
        self.handle = h.value
        if exact is not None:
            try:
                self.set_exact(exact)
            except Exception:
                self.destroy()
                raise
        n = C.c_int()
        check(lib.mvg_comm_local_count(comm.handle, C.byref(n)), "mvg_comm_local_count")
        self.nlocal = n.value

    @property
    def name(self) -> str:
        return ALG_NAMES[self.alg]

    def shard(self, i: int = 0) -> Shard:
        s = Shard()
        check(lib.mvg_engine_shard(self.handle, i, C.byref(s)), "mvg_engine_shard")
        return s

    def stream(self, i: int = 0) -> int:
        p = C.c_void_p()
        check(lib.mvg_engine_stream(self.handle, i, C.byref(p)), "mvg_engine_stream")
        return p.value or 0

    def is_root(self) -> bool:
        return any(self.shard(i).rank == 0 for i in range(self.nlocal))

    def distribute(self, A: np.ndarray | None, x: np.ndarray | None) -> None:
        """Root's host A, x -> every device's shard (A, x may be None off the root)."""
        pa = np.ascontiguousarray(A, dtype=np.float64).ctypes.data if A is not None else None
        px = np.ascontiguousarray(x, dtype=np.float64).ctypes.data if x is not None else None
        self._keep = (A, x)
        check(lib.mvg_engine_distribute(self.handle, pa, px), "mvg_engine_distribute")

    def distribute_shared(self, A: np.ndarray, x: np.ndarray) -> None:
        """Every rank passes the root's A, x mapped from shared host memory; each GPU pulls its
        own shard over its own PCIe link, concurrently."""
        A = np.ascontiguousarray(A, dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=np.float64)
        self._keep = (A, x)
        check(lib.mvg_engine_distribute_shared(self.handle, A.ctypes.data, x.ctypes.data),
              "mvg_engine_distribute_shared")

    def fill_synth(self, seed_a: int = SEED_A, seed_x: int = SEED_X) -> None:
        check(lib.mvg_engine_fill_synth(self.handle, seed_a, seed_x), "mvg_engine_fill_synth")

    def multiply(self) -> None:
        check(lib.mvg_engine_multiply(self.handle), "mvg_engine_multiply")

    def sync(self) -> None:
        check(lib.mvg_engine_sync(self.handle), "mvg_engine_sync")

    def collect(self) -> np.ndarray | None:
        """y on the root (None elsewhere)."""
        if not self.is_root():
            check(lib.mvg_engine_sync(self.handle), "mvg_engine_sync")
            return None
        y = np.empty(max(self.R, 1), dtype=np.float64)
        check(lib.mvg_engine_collect(self.handle, y.ctypes.data), "mvg_engine_collect")
        return y[: self.R]

    def set_exact(self, on: bool) -> None:
        check(lib.mvg_engine_set_exact(self.handle, int(bool(on))), "mvg_engine_set_exact")

    def set_overlap(self, chunks: int) -> None:
        """Distribute in `chunks` row chunks, each chunk's GEMV behind its copy (0/1 = off)."""
        check(lib.mvg_engine_set_overlap(self.handle, int(chunks)), "mvg_engine_set_overlap")

    @property
    def exact(self) -> bool:
        v = C.c_int()
        check(lib.mvg_engine_exact(self.handle, C.byref(v)), "mvg_engine_exact")
        return bool(v.value)

    def exact_panel_width(self, i: int = 0) -> int:
        """Panel width of local shard i's column-panel copy in exact mode (0: row-major kernels)."""
        v = C.c_int64()
        check(lib.mvg_engine_exact_panels(self.handle, i, C.byref(v)), "mvg_engine_exact_panels")
        return v.value

    def kernel_timing(self, every: int) -> None:
        """Bracket every `every`-th multiply's GEMV with HIP events (0 = off); -1 times spans of
        back-to-back multiplies, one event pair from the first GEMV to the next sync."""
        check(lib.mvg_engine_kernel_timing(self.handle, int(every)), "mvg_engine_kernel_timing")

    def kernel_ms(self) -> KernelTiming:
        ms, n = C.c_double(), C.c_int64()
        check(lib.mvg_engine_kernel_ms(self.handle, C.byref(ms), C.byref(n)), "mvg_engine_kernel_ms")
        return KernelTiming(ms.value, n.value)

    def destroy(self) -> None:
        if self.handle:
            lib.mvg_engine_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()


def device_count() -> int:
    n = C.c_int()
    check(lib.mvg_device_count(C.byref(n)), "mvg_device_count")
    return n.value


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v else default
