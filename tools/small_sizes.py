"""Per-multiply cost at the reference's small test.sh sizes (development tool).

For each shape: device-resident engine multiplies back to back (host wall per multiply), the
same with the GEMV kernel alone through mvg_gemv, and a no-op baseline (hipLaunch of the zero
kernel via k = 0). Prints one JSON line per shape.
"""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

SHAPES = [(600, 600), (1800, 1800), (4200, 4200), (10200, 10200), (120, 60000), (1200, 60000)]
ITERS = 2000


def main():
    alg = sys.argv[1] if len(sys.argv) > 1 else "rowwise"
    comm = mm.Comm.init_all([0])
    for R, C in SHAPES:
        eng = mm.Multiplier(alg, R, C, comm)
        eng.fill_synth()
        eng.sync()
        for _ in range(50):
            eng.multiply()
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(ITERS):
            eng.multiply()
        t_enq = time.perf_counter() - t0
        eng.sync()
        t_all = time.perf_counter() - t0
        eng.kernel_timing(1)
        for _ in range(200):
            eng.multiply()
        kt = eng.kernel_ms()
        eng.kernel_timing(0)
        out = {"alg": alg, "R": R, "C": C, "us_per_multiply": round(t_all / ITERS * 1e6, 2),
               "host_enqueue_us": round(t_enq / ITERS * 1e6, 2), "kernel_us_events": round(kt.avg_ms * 1e3, 2),
               "GBps": round(8 * (R * C + R + C) / (t_all / ITERS) / 1e9, 1)}
        print(json.dumps(out), flush=True)
        eng.destroy()
    comm.destroy()


if __name__ == "__main__":
    main()
