"""Where does the row-major exact GEMV lose time inside the engine? (development tool, one MI355X)

    python tools/probes/engine_exact_probe.py [M] [K] [launches]

The same kernels (mvg_gemv tree, mvg_gemv_exact) on the same shape, three ways, interleaved twice:
  engine : mm.Multiplier (fill_synth, MVG_NO_PANELS=1), kernel time from its HIP events;
  hipmalloc: A, x, y from mvg_malloc (the engine's allocator), launched directly;
  torch  : A, x, y from torch's caching allocator, launched directly (the variant sweeps' setup).
One JSON object per (way, kernel).
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MVG_NO_PANELS"] = "1"
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def timed(fn, n, s):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def raw(M, K, n, A, x, y, s):
    return {"tree": timed(lambda: lib.mvg_gemv(A, K, x, y, M, K, s), n, s),
            "exact": timed(lambda: lib.mvg_gemv_exact(A, K, x, y, M, K, s), n, s)}


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    # torch buffers
    tA = torch.empty(M * K, dtype=torch.float64, device="cuda:0")
    tx = torch.empty(K, dtype=torch.float64, device="cuda:0")
    ty = torch.empty(M, dtype=torch.float64, device="cuda:0")
    # engine-allocator buffers
    ptrs = []
    for count in (M * K, K, M):
        p = C.c_void_p()
        check(lib.mvg_malloc(C.byref(p), count * 8), "mvg_malloc")
        ptrs.append(p.value)
    hA, hx, hy = ptrs
    for A, x in ((tA.data_ptr(), tx.data_ptr()), (hA, hx)):
        check(lib.mvg_synth_fill_device(A, K, M, K, 0, 0, K, 42, s), "fill")
        check(lib.mvg_synth_fill_device(x, K, 1, K, 0, 0, K, 4242, s), "fill")
    comm = mm.Comm.init_all([0])
    eng = mm.Multiplier("rowwise", M, K, comm)
    eng.fill_synth()
    eng.sync()
    for _ in range(2):
        for way in ("engine", "hipmalloc", "torch"):
            if way == "engine":
                out = {}
                for exact in (False, True):
                    eng.set_exact(exact)
                    for _ in range(3):
                        eng.multiply()
                    eng.kernel_timing(1)
                    for _ in range(n):
                        eng.multiply()
                    out["exact" if exact else "tree"] = eng.kernel_ms().avg_ms * 1e3
                    eng.kernel_timing(0)
                eng.set_exact(False)
            elif way == "hipmalloc":
                out = raw(M, K, n, hA, hx, hy, s)
            else:
                out = raw(M, K, n, tA.data_ptr(), tx.data_ptr(), ty.data_ptr(), s)
            for k, v in out.items():
                res.setdefault((way, k), []).append(round(v, 2))
    for (way, k), v in res.items():
        print(json.dumps({"M": M, "K": K, "way": way, "kernel": k, "us": v}), flush=True)
    eng.destroy()
    comm.destroy()
    for p in ptrs:
        lib.mvg_free(p)


if __name__ == "__main__":
    main()
