"""End-to-end time (root's host A, x -> distribute -> multiply -> y on the host) with the
chunked distribution (mvg_engine_set_overlap) at several chunk counts, one GPU (development tool).

    python tools/probes/overlap_probe.py [R] [C] [iters]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import lib  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    A = mm.synth_host(R, C, 42)
    x = mm.synth_host(1, C, 4242)[0]
    assert lib.mvg_host_register(A.ctypes.data, A.nbytes) == 0
    comm = mm.Comm.init_all([0])
    ref = None
    for alg in ("rowwise", "colwise"):
        for exact in (False, True):
            with mm.Multiplier(alg, R, C, comm, exact=exact) as e:
                for chunks in (0, 2, 4, 8, 16, 32):
                    e.set_overlap(chunks)
                    e.distribute(A, x)
                    e.multiply()
                    y = e.collect()
                    if ref is None or chunks == 0:
                        ref = y
                    same = bool(np.array_equal(y, ref))
                    ts = []
                    for _ in range(iters):
                        t0 = time.perf_counter()
                        e.distribute(A, x)
                        e.multiply()
                        e.collect()
                        ts.append(time.perf_counter() - t0)
                    print(json.dumps({"R": R, "C": C, "alg": alg, "exact": exact, "chunks": chunks,
                                      "mean_ms": round(1e3 * float(np.mean(ts)), 4),
                                      "min_ms": round(1e3 * float(np.min(ts)), 4),
                                      "y_equal_to_unchunked": same}), flush=True)
    lib.mvg_host_unregister(A.ctypes.data)
    comm.destroy()


if __name__ == "__main__":
    main()
