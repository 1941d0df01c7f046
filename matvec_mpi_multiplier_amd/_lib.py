"""ctypes binding of libmatvec_gpu.so (the C-ABI declared in include/matvec_gpu.h).

The library is the product: there is no Python or CPU fallback for any compute call. If the
shared object is missing this module raises at import time with the build command to run.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MVG_LIB: another build of the same library (the sanitizer build, `make asan`)
LIB_PATH = os.environ.get("MVG_LIB") or os.path.join(_HERE, "libmatvec_gpu.so")

MVG_OK = 0
MVG_E_INVALID = -1
MVG_E_INDIVISIBLE = -2
MVG_E_HIP = -3
MVG_E_RCCL = -4
MVG_E_IO = -5
MVG_E_NOMEM = -6
MVG_E_STATE = -7

ALG_ROWWISE, ALG_COLWISE, ALG_BLOCKWISE = 0, 1, 2
ALG_NAMES = {ALG_ROWWISE: "rowwise", ALG_COLWISE: "colwise", ALG_BLOCKWISE: "blockwise"}
ALG_BY_NAME = {v: k for k, v in ALG_NAMES.items()}

SEED_A = 42
SEED_X = 4242
UNIQUE_ID_BYTES = 128


class MvgError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str):
        self.code = code
        super().__init__(f"{where} failed ({code}): {detail}")


class IndivisibleError(MvgError):
    """Shape does not split over the rank count (the reference's "ERROR!!!" case)."""


class Shard(C.Structure):
    """mvg_shard: the slice of the global problem one rank owns."""

    _fields_ = [
        ("alg", C.c_int), ("nranks", C.c_int), ("rank", C.c_int),
        ("grid_rows", C.c_int), ("grid_cols", C.c_int), ("grid_r", C.c_int), ("grid_c", C.c_int),
        ("R", C.c_int64), ("C", C.c_int64),
        ("row_off", C.c_int64), ("col_off", C.c_int64), ("n_rows", C.c_int64), ("n_cols", C.c_int64),
        ("y_off", C.c_int64), ("y_len", C.c_int64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class XStep(C.Structure):
    """mvg_xstep: one collective of the exchange schedule (mvg_plan_exchange)."""

    _fields_ = [
        ("op", C.c_int), ("comm", C.c_int), ("color", C.c_int), ("key", C.c_int),
        ("member", C.c_int), ("root", C.c_int), ("src", C.c_int), ("dst", C.c_int),
        ("count", C.c_int64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class XCall(C.Structure):
    """mvg_xcall: one call of the single-process exchange (mvg_debug_trace_exchange)."""

    _fields_ = [
        ("group", C.c_int), ("kind", C.c_int), ("rank", C.c_int), ("comm", C.c_int), ("color", C.c_int),
        ("key", C.c_int), ("root", C.c_int), ("src", C.c_int), ("dst", C.c_int), ("count", C.c_int64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


X_GATHER, X_REDUCE = 0, 1
X_WORLD, X_ROW, X_COL = 0, 1, 2
X_BUF_PART, X_BUF_ROW, X_BUF_Y, X_BUF_GATHERED = 0, 1, 2, 3
XCALL_SPLIT, XCALL_GATHER, XCALL_REDUCE, XCALL_COMBINE = 0, 1, 2, 3
MAX_XSTEPS = 4

_p = C.c_void_p
_i64 = C.c_int64
_dp = C.POINTER(C.c_double)

# name -> (restype, argtypes); the order follows include/matvec_gpu.h
SIGNATURES = {
    "mvg_version": (C.c_char_p, []),
    "mvg_strerror": (C.c_char_p, [C.c_int]),
    "mvg_last_error": (C.c_char_p, []),
    "mvg_runtime_versions": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mvg_runtime_path": (C.c_char_p, [C.c_int]),
    "mvg_grid_shape": (C.c_int, [_i64, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mvg_plan_shard": (C.c_int, [C.c_int, _i64, _i64, C.c_int, C.c_int, C.POINTER(Shard)]),
    "mvg_plan_exchange": (C.c_int, [C.c_int, _i64, _i64, C.c_int, C.c_int, C.c_int, C.POINTER(XStep), C.c_int,
                                     C.POINTER(C.c_int)]),
    "mvg_synth_value": (C.c_double, [C.c_uint64, C.c_uint64]),
    "mvg_synth_fill_host": (C.c_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, C.c_uint64]),
    "mvg_synth_fill_device": (C.c_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, C.c_uint64, _p]),
    "mvg_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "mvg_set_device": (C.c_int, [C.c_int]),
    "mvg_malloc": (C.c_int, [C.POINTER(_p), C.c_size_t]),
    "mvg_free": (C.c_int, [_p]),
    "mvg_memcpy_h2d": (C.c_int, [_p, _p, C.c_size_t, _p]),
    "mvg_memcpy_d2h": (C.c_int, [_p, _p, C.c_size_t, _p]),
    "mvg_stream_sync": (C.c_int, [_p]),
    "mvg_host_register": (C.c_int, [_p, C.c_size_t]),
    "mvg_host_unregister": (C.c_int, [_p]),
    "mvg_device_numa_node": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "mvg_host_first_touch": (C.c_int, [_p, C.c_size_t, C.c_int]),
    "mvg_gemv": (C.c_int, [_p, _i64, _p, _p, _i64, _i64, _p]),
    "mvg_gemv_variant": (C.c_int, [_p, _i64, _p, _p, _i64, _i64, C.c_int, _p]),
    "mvg_gemv_variant_count": (C.c_int, []),
    "mvg_gemv_variant_name": (C.c_char_p, [C.c_int]),
    "mvg_gemv_auto_variant": (C.c_int, [_i64, _i64, _i64]),
    "mvg_gemv_multi": (C.c_int, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, C.c_int, _p]),
    "mvg_gemv_multi_variant": (C.c_int, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, C.c_int, C.c_int, _p]),
    "mvg_gemv_multi_variant_count": (C.c_int, []),
    "mvg_gemv_multi_auto_variant": (C.c_int, [_i64, _i64, _i64, _i64, C.c_int]),
    "mvg_gemv_multi_variant_name": (C.c_char_p, [C.c_int]),
    "mvg_gemv_exact": (C.c_int, [_p, _i64, _p, _p, _i64, _i64, _p]),
    "mvg_multiply_std_rowwise": (C.c_int, [_p, _p, _i64, _i64, _p, C.c_int]),
    "mvg_gemv_exact_variant": (C.c_int, [_p, _i64, _p, _p, _i64, _i64, C.c_int, _p]),
    "mvg_gemv_exact_variant_count": (C.c_int, []),
    "mvg_gemv_exact_auto_variant": (C.c_int, [_i64, _i64, _i64]),
    "mvg_debug_set_cu_count": (C.c_int, [C.c_int]),
    "mvg_debug_trace_exchange": (C.c_int, [C.c_int, _i64, _i64, C.c_int, C.c_int, C.POINTER(XCall), C.c_int,
                                           C.POINTER(C.c_int)]),
    "mvg_debug_set_exact_even_lds": (C.c_int, [_i64]),
    "mvg_gemv_exact_even_refused": (C.c_int, [C.c_int]),
    "mvg_gemv_exact_variant_name": (C.c_char_p, [C.c_int]),
    "mvg_gemv_exact_panels": (C.c_int, [_p, _i64, _i64, _p, _p, _i64, _i64, C.c_int, _p]),
    "mvg_panel_relayout": (C.c_int, [_p, _i64, _i64, _i64, _p, _i64, _i64, _p]),
    "mvg_exact_panel_width": (_i64, [_i64, _i64]),
    "mvg_gemv_exact_panel_variant_count": (C.c_int, []),
    "mvg_gemv_exact_panel_auto_variant": (C.c_int, [_i64, _i64]),
    "mvg_gemv_exact_panel_variant_name": (C.c_char_p, [C.c_int]),
    "mvg_stream_read": (C.c_int, [_p, _i64, _p, _p]),
    "mvg_comm_unique_id": (C.c_int, [C.c_char_p]),
    "mvg_comm_init_all": (C.c_int, [C.POINTER(_p), C.c_int, C.POINTER(C.c_int)]),
    "mvg_comm_init_rank": (C.c_int, [C.POINTER(_p), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mvg_comm_size": (C.c_int, [_p, C.POINTER(C.c_int)]),
    "mvg_comm_local_count": (C.c_int, [_p, C.POINTER(C.c_int)]),
    "mvg_comm_local_rank": (C.c_int, [_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mvg_comm_destroy": (C.c_int, [_p]),
    "mvg_engine_create": (C.c_int, [C.POINTER(_p), C.c_int, _i64, _i64, _p]),
    "mvg_engine_shard": (C.c_int, [_p, C.c_int, C.POINTER(Shard)]),
    "mvg_engine_distribute": (C.c_int, [_p, _p, _p]),
    "mvg_engine_distribute_shared": (C.c_int, [_p, _p, _p]),
    "mvg_engine_fill_synth": (C.c_int, [_p, C.c_uint64, C.c_uint64]),
    "mvg_engine_multiply": (C.c_int, [_p]),
    "mvg_engine_sync": (C.c_int, [_p]),
    "mvg_engine_collect": (C.c_int, [_p, _p]),
    "mvg_engine_stream": (C.c_int, [_p, C.c_int, C.POINTER(_p)]),
    "mvg_engine_kernel_timing": (C.c_int, [_p, C.c_int]),
    "mvg_engine_kernel_ms": (C.c_int, [_p, C.POINTER(C.c_double), C.POINTER(_i64)]),
    "mvg_engine_destroy": (C.c_int, [_p]),
    "mvg_engine_set_exact": (C.c_int, [_p, C.c_int]),
    "mvg_engine_exact": (C.c_int, [_p, C.POINTER(C.c_int)]),
    "mvg_engine_exact_panels": (C.c_int, [_p, C.c_int, C.POINTER(_i64)]),
    "mvg_engine_set_overlap": (C.c_int, [_p, C.c_int]),
    "mvg_matrix_filename": (C.c_int, [_i64, _i64, C.c_char_p, C.c_size_t]),
    "mvg_vector_filename": (C.c_int, [_i64, C.c_char_p, C.c_size_t]),
    "mvg_load_matr": (C.c_int, [C.c_char_p, _i64, _i64, _p]),
    "mvg_write_matr_bin": (C.c_int, [C.c_char_p, _p, _i64, _i64]),
    "mvg_load_vec": (C.c_int, [C.c_char_p, _i64, _p]),
    "mvg_write_vec": (C.c_int, [C.c_char_p, _p, _i64]),
    "mvg_write_matr_synth": (C.c_int, [C.c_char_p, _i64, _i64, C.c_uint64]),
}


def _torch_first() -> None:
    """PyTorch's ROCm wheel bundles its own HIP and HSA runtimes (libamdhip64.so, soname
    libamdhip64.so.7, HIP 7.0). Loaded after this library, they make a second HIP + HSA runtime
    in the process, and two HSA runtimes cannot both open the GPU: whichever initialises second
    finds "no ROCm-capable device" (profiles/r05/torch_order/). Loaded first, PyTorch's copy
    satisfies this library's dependency on libamdhip64.so.7 (same soname), so the process has one
    HIP runtime that both use, in any order, with the tree kernel's time unchanged. So when
    PyTorch is installed it is imported before the library is loaded; MVG_NO_TORCH=1 skips that
    (a process that never uses PyTorch's GPU side then runs on /opt/rocm's runtime). PyTorch's
    RCCL (librccl.so.1, 2.26.6 in this image) binds the same way, so a Python process runs the
    library's collectives on it; runtime_info() says which copies a process runs on."""
    if os.environ.get("MVG_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    except Exception as exc:  # a broken install (a missing .so: OSError, ...): the library's own runtime
        import sys

        print(f"matvec_mpi_multiplier_amd: importing torch failed ({type(exc).__name__}: {str(exc)[:200]}); "
              "the library runs on its own HIP runtime (/opt/rocm)", file=sys.stderr)


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: the HIP library is required (no CPU fallback). "
            "Build it with `make -C <repo>` or `python -c 'import __graft_entry__ as g; g.build()'`."
        )
    _torch_first()
    lib = C.CDLL(LIB_PATH)  # RTLD_LOCAL: a global RCCL ahead of torch's double-frees at exit
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, where: str) -> None:
    if rc != MVG_OK:
        detail = lib.mvg_last_error().decode(errors="replace")
        cls = IndivisibleError if rc == MVG_E_INDIVISIBLE else MvgError
        raise cls(rc, where, detail)


def mapped_runtimes(maps_lines) -> dict:
    """The files of the HIP runtime and RCCL mapped into a process, from its /proc/<pid>/maps
    lines: {"libamdhip64": [paths], "librccl": [paths]} (more than one path per library: two
    copies are loaded)."""
    out: dict = {"libamdhip64": set(), "librccl": set()}
    for line in maps_lines:
        parts = line.split(None, 5)
        if len(parts) < 6:
            continue
        path = parts[5].strip()
        base = os.path.basename(path)
        for key in out:
            if base.startswith(key + ".so"):
                out[key].add(path)
    return {k: sorted(v) for k, v in out.items()}


def rccl_version_text(code: int) -> str:
    """ncclGetVersion's code as X.Y.Z (NCCL_VERSION_CODE: X*10000 + Y*100 + Z since 2.9)."""
    return f"{code // 10000}.{code // 100 % 100}.{code % 100}" if code >= 10000 else f"{code // 1000}.{code // 100 % 10}.{code % 100}"


def runtime_info(hip_version: bool = True) -> dict:
    """Which HIP runtime and RCCL this process's library calls go to (mvg_runtime_versions /
    mvg_runtime_path: the copies the library resolved), every copy mapped into the process
    (/proc/self/maps), and whether they are PyTorch's bundled ones or /opt/rocm's."""
    r, h = C.c_int(0), C.c_int(0)
    rc = lib.mvg_runtime_versions(C.byref(r), C.byref(h) if hip_version else None)
    hip_path = lib.mvg_runtime_path(0).decode(errors="replace")
    rccl_path = lib.mvg_runtime_path(1).decode(errors="replace")
    try:
        with open("/proc/self/maps") as f:
            mapped = mapped_runtimes(f)
    except OSError:
        mapped = None

    def origin(p):
        return "pytorch" if "/torch/lib/" in p else "rocm" if "/rocm" in p else ("unknown" if p else None)

    return {"rccl_version": rccl_version_text(r.value) if rc == MVG_OK and r.value else None,
            "rccl_version_code": r.value if rc == MVG_OK else None,
            "hip_runtime_version": h.value if rc == MVG_OK and hip_version else None,
            "hip_path": hip_path, "rccl_path": rccl_path,
            "hip_origin": origin(hip_path), "rccl_origin": origin(rccl_path), "mapped": mapped}


def ptr(a) -> int:
    """Address of a numpy array's data (host) as an int for ctypes."""
    return a.ctypes.data
