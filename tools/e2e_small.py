"""Where the end-to-end time of a small multiply goes (development tool).

    python tools/e2e_small.py [--spin] [--pin-xy] [--iters 200]

One GPU, the executables' loop (sync; distribute A, x from the root's host memory; multiply;
collect y; sync) on the reference's small test.sh sizes, each phase timed on the host with a
stream synchronize after it, then the whole iteration timed without the intermediate syncs.
--spin sets hipDeviceScheduleSpin before the runtime starts; --pin-xy page-locks x and y too
(A is always page-locked, as in the executables).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--pin-xy", action="store_true")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--alg", default="rowwise")
    args = ap.parse_args()
    if args.spin:
        hip = C.CDLL("libamdhip64.so")
        assert hip.hipSetDeviceFlags(1) == 0  # hipDeviceScheduleSpin
    from matvec_mpi_multiplier_amd import multiplier as mm
    from matvec_mpi_multiplier_amd._lib import lib, check

    comm = mm.Comm.init_all([0])
    for n in (600, 1200, 1800, 3000, 4200):
        eng = mm.Multiplier(args.alg, n, n, comm)
        A = mm.synth_host(n, n, 42)
        x = mm.synth_host(1, n, 4242)[0].copy()
        y = np.empty(n)
        check(lib.mvg_host_register(A.ctypes.data, A.nbytes), "reg")
        if args.pin_xy:
            check(lib.mvg_host_register(x.ctypes.data, x.nbytes), "reg x")
            check(lib.mvg_host_register(y.ctypes.data, y.nbytes), "reg y")
        h = eng.handle
        ph = {"distribute": [], "multiply": [], "collect": [], "whole": []}
        for it in range(args.iters + 10):
            check(lib.mvg_engine_sync(h), "sync")
            t0 = time.perf_counter()
            check(lib.mvg_engine_distribute(h, A.ctypes.data, x.ctypes.data), "dist")
            check(lib.mvg_engine_sync(h), "sync")
            t1 = time.perf_counter()
            check(lib.mvg_engine_multiply(h), "mul")
            check(lib.mvg_engine_sync(h), "sync")
            t2 = time.perf_counter()
            check(lib.mvg_engine_collect(h, y.ctypes.data), "collect")
            t3 = time.perf_counter()
            check(lib.mvg_engine_sync(h), "sync")
            t4 = time.perf_counter()
            check(lib.mvg_engine_distribute(h, A.ctypes.data, x.ctypes.data), "dist")
            check(lib.mvg_engine_multiply(h), "mul")
            check(lib.mvg_engine_collect(h, y.ctypes.data), "collect")
            check(lib.mvg_engine_sync(h), "sync")
            t5 = time.perf_counter()
            if it >= 10:
                for k, dt in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t5 - t4)):
                    ph[k].append(dt * 1e6)
        out = {"alg": args.alg, "n": n, "spin": args.spin, "pin_xy": args.pin_xy, 
               "A_h2d_GBps_median": round(A.nbytes / (np.median(ph["distribute"]) * 1e-6) / 1e9, 1)}
        for k, v in ph.items():
            out[k + "_us_median"] = round(float(np.median(v)), 1)
            out[k + "_us_mean"] = round(float(np.mean(v)), 1)
        print(json.dumps(out), flush=True)
        if args.pin_xy:
            lib.mvg_host_unregister(x.ctypes.data)
            lib.mvg_host_unregister(y.ctypes.data)
        lib.mvg_host_unregister(A.ctypes.data)
        eng.destroy()
    comm.destroy()


if __name__ == "__main__":
    main()
