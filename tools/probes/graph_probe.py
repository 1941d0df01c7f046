"""Does a HIP graph lower the per-multiply cost of small, launch-bound GEMVs? (development tool)

For a few small shapes: n back-to-back mvg_gemv launches on one stream (eager) against n
hipGraphLaunch of a graph captured from one mvg_gemv, and against one graph holding 20 GEMVs
(per-GEMV cost), all timed on the host around a stream synchronize."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

hip = C.CDLL("libamdhip64.so")
for f in ("hipStreamBeginCapture", "hipStreamEndCapture", "hipGraphInstantiate", "hipGraphLaunch",
          "hipStreamSynchronize", "hipStreamCreate"):
    getattr(hip, f).restype = C.c_int


def main():
    s = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(s)) == 0
    for n in (600, 1800, 4200):
        dA, dx, dy = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check(lib.mvg_malloc(C.byref(dA), n * n * 8), "m")
        check(lib.mvg_malloc(C.byref(dx), n * 8), "m")
        check(lib.mvg_malloc(C.byref(dy), n * 8), "m")
        check(lib.mvg_synth_fill_device(dA, n, n, n, 0, 0, n, 42, s), "f")
        check(lib.mvg_synth_fill_device(dx, n, 1, n, 0, 0, n, 4242, s), "f")

        def gemv():
            return lib.mvg_gemv(dA, n, dx, dy, n, n, s)

        def graph_of(k):
            g, ge = C.c_void_p(), C.c_void_p()
            assert hip.hipStreamBeginCapture(s, 0) == 0
            for _ in range(k):
                check(gemv(), "gemv")
            assert hip.hipStreamEndCapture(s, C.byref(g)) == 0
            assert hip.hipGraphInstantiate(C.byref(ge), g, None, None, 0) == 0
            return ge

        g1, g20 = graph_of(1), graph_of(20)
        out = {"n": n}
        reps = 2000
        for name, fn, per in (("eager", gemv, 1), ("graph1", lambda: hip.hipGraphLaunch(g1, s), 1),
                              ("graph20", lambda: hip.hipGraphLaunch(g20, s), 20)):
            for _ in range(50):
                fn()
            hip.hipStreamSynchronize(s)
            t = time.perf_counter()
            for _ in range(reps // per):
                fn()
            t_enq = time.perf_counter() - t
            hip.hipStreamSynchronize(s)
            t_all = time.perf_counter() - t
            out[name + "_us_per_gemv"] = round(t_all / reps * 1e6, 2)
            out[name + "_enqueue_us_per_gemv"] = round(t_enq / reps * 1e6, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
