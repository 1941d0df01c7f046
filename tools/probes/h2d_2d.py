"""Strided (column-strip / block) host->device copies vs contiguous ones (development tool).

The column and block splits distribute sub-windows of the root's row-major A: hipMemcpy2DAsync
with host pitch C and width C/P (engine.cpp h2d_region). This times that copy, for several strip
widths, against a contiguous copy of the same bytes, from page-locked host memory."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                 C.c_int, C.c_void_p]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]


def timed(fn, reps=4):
    ts = []
    for _ in range(reps):
        hip.hipDeviceSynchronize()
        t = time.perf_counter()
        assert fn() == 0
        hip.hipDeviceSynchronize()
        ts.append(time.perf_counter() - t)
    return min(ts[1:])


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    Cn = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    A = np.empty((R, Cn))
    check(lib.mvg_synth_fill_host(A.ctypes.data, Cn, R, Cn, 0, 0, Cn, 42), "fill")
    check(lib.mvg_host_register(A.ctypes.data, A.nbytes), "register")
    d = C.c_void_p()
    check(lib.mvg_malloc(C.byref(d), A.nbytes // 2), "malloc")
    for P in (2, 4, 8, 16):
        w = Cn // P
        nbytes = R * w * 8
        t2 = timed(lambda: hip.hipMemcpy2DAsync(d, w * 8, A.ctypes.data + (P - 1) * w * 8, Cn * 8, w * 8, R, 1, None))
        t1 = timed(lambda: hip.hipMemcpyAsync(d, A.ctypes.data, nbytes, 1, None))
        print(json.dumps({"R": R, "C": Cn, "strip_cols": w, "bytes": nbytes,
                          "strided_GBps": round(nbytes / t2 / 1e9, 1), "contiguous_GBps": round(nbytes / t1 / 1e9, 1)}),
              flush=True)
    lib.mvg_host_unregister(A.ctypes.data)


if __name__ == "__main__":
    main()
