"""Text loader throughput (development tool): writes the reference's text format for an R x C
synthetic matrix (mvg_write_matr_synth, "%.4f") into a scratch directory, then times
mvg_load_matr on it at the given thread counts (MVG_THREADS; best of 3), checking that every
thread count reads the same values (a checksum). One JSON line per thread count.

    python tools/load_bench.py [R] [C] [threads,threads,...] [scratch dir]
"""
import json
import os
import subprocess
import sys


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    Cn = int(sys.argv[2]) if len(sys.argv) > 2 else R
    threads = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "1,4,16").split(",")]
    d = sys.argv[4] if len(sys.argv) > 4 else "/tmp/mvg_load_bench"
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"matrix_{R}_{Cn}.txt")
    if not os.path.exists(path):
        check(lib.mvg_write_matr_synth(path.encode(), R, Cn, 42), "write")
    size = os.path.getsize(path)
    ref = None
    for nt in threads:
        # each thread count in a child process of its own (a fresh heap for the 8-B values)
        code = ("import ctypes as C, sys, time, numpy as np; sys.path.insert(0, %r);"
                "from matvec_mpi_multiplier_amd._lib import lib, check;"
                "A = np.empty(%d); ts = []\n"
                "for _ in range(3):\n"
                "    t = time.perf_counter(); check(lib.mvg_load_matr(%r.encode(), %d, %d, A.ctypes.data_as(C.POINTER(C.c_double))), 'load'); ts.append(time.perf_counter() - t)\n"
                "print(min(ts), float(A[:1000003].sum()))") % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), R * Cn, d, R, Cn)
        out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MVG_THREADS=str(nt), MVG_BIN_CACHE="0"),
                             capture_output=True, text=True, check=True).stdout.split()
        best, cs = float(out[0]), float(out[1])
        ref = cs if ref is None else ref
        print(json.dumps({"R": R, "C": Cn, "bytes": size, "threads": nt, "best_s": round(best, 4),
                          "GBps": round(size / best / 1e9, 3), "checksum_agrees": cs == ref}), flush=True)


if __name__ == "__main__":
    main()
