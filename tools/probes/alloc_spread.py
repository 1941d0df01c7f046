"""Placement spread probe (development tool): the config-2 GEMV (16384^2, auto variant) and the
read-only stream kernel on several freshly allocated 2 GiB buffers of one process, to tell
allocation placement effects (spread across buffers) from box effects (spread across runs).

    python tools/probes/alloc_spread.py [--buffers 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def timed(fn, reps=20):
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=8)
    args = ap.parse_args()
    n = 16384
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    sink = torch.zeros(256 * 16 * 256, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(x.data_ptr(), n, 1, n, 0, 0, n, 4242, s), "fill x")
    bufs = []
    for b in range(args.buffers):
        A = torch.empty(n * n, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(A.data_ptr(), n, n, n, 0, 0, n, 42, s), "fill A")
        bufs.append(A)
        g = timed(lambda: lib.mvg_gemv(A.data_ptr(), n, x.data_ptr(), y.data_ptr(), n, n, s))
        r = timed(lambda: lib.mvg_stream_read(A.data_ptr(), n * n, sink.data_ptr(), s))
        print(json.dumps({"buffer": b, "addr_GiB": round(A.data_ptr() / 2**30, 1),
                          "gemv_us": round(g * 1e3, 1), "gemv_TBps": round(8 * (n * n + 2 * n) / g / 1e9, 3),
                          "stream_TBps": round(8 * n * n / r / 1e9, 3)}), flush=True)
    # the first buffer again, after all the others exist
    A = bufs[0]
    g = timed(lambda: lib.mvg_gemv(A.data_ptr(), n, x.data_ptr(), y.data_ptr(), n, n, s))
    print(json.dumps({"buffer": "0-again", "gemv_TBps": round(8 * (n * n + 2 * n) / g / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
