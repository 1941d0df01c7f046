"""What the first H2D of a freshly page-locked buffer pays (development tool).

Times, in one fresh process: an H2D of NBYTES from a page-locked scratch buffer (hipHostMalloc),
then the first and second H2D of the same size from a hipHostRegister'ed numpy buffer, then the
first H2D from a second registered buffer. Splits the one-time cost into a per-process part
(copy path bring-up) and a per-buffer part (first DMA over newly registered pages)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def main():
    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 600 * 600 * 8
    d = C.c_void_p()
    check(lib.mvg_malloc(C.byref(d), nbytes), "malloc")
    assert hip.hipMemset(d, 0, C.c_size_t(nbytes)) == 0
    out = {"bytes": nbytes}

    def h2d(src, tag):
        hip.hipDeviceSynchronize()
        t = time.perf_counter()
        check(lib.mvg_memcpy_h2d(d.value, src, nbytes, None), "h2d")
        hip.hipDeviceSynchronize()
        out[tag] = round((time.perf_counter() - t) * 1e6, 1)

    if "--no-scratch" not in sys.argv:
        p = C.c_void_p()
        assert hip.hipHostMalloc(C.byref(p), C.c_size_t(nbytes), 0) == 0
        h2d(p.value, "scratch_first_us")
        h2d(p.value, "scratch_second_us")
    a = np.ones(nbytes // 8)
    b = np.ones(nbytes // 8)
    t = time.perf_counter()
    check(lib.mvg_host_register(a.ctypes.data, a.nbytes), "reg")
    out["register_us"] = round((time.perf_counter() - t) * 1e6, 1)
    check(lib.mvg_host_register(b.ctypes.data, b.nbytes), "reg")
    h2d(a.ctypes.data, "registered_first_us")
    h2d(a.ctypes.data, "registered_second_us")
    h2d(b.ctypes.data, "other_registered_first_us")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
