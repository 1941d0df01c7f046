"""Is the tree kernel's process-to-process spread (293 vs 301 µs at config 2, profiles/r05/m5d)
a property of the stream / hardware queue a launch goes to? (development probe)

    python tools/probes/stream_probe.py [M] [K] [streams] [launches]

One 2 GiB A (config 2) on the device; the same mvg_gemv launched back to back on each of
`streams` HIP streams in turn (PyTorch's streams: the package loads PyTorch first, so they are
the library's runtime's streams too), timed with one event pair per stream around `launches`
launches. Prints one JSON line: µs per launch per stream, in creation order.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    import torch

    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    ns = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 100
    torch.cuda.set_device(0)
    dA, dx, dy = mm.DeviceBuffer(M * K), mm.DeviceBuffer(K), mm.DeviceBuffer(M)
    check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, None), "fill A")
    check(lib.mvg_synth_fill_device(dx.ptr, K, 1, K, 0, 0, K, 4242, None), "fill x")
    check(lib.mvg_stream_sync(None), "sync")
    streams = [torch.cuda.Stream() for _ in range(ns)]
    out = {"M": M, "K": K, "launches": n, "us_by_stream": [], "default_stream_us": None}

    def timed(st):
        h = st.cuda_stream if st is not None else None
        for _ in range(30):
            check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, h), "gemv")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if st is not None:
            e0.record(st)
        else:
            check(lib.mvg_stream_sync(None), "sync")
        for _ in range(n):
            check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, h), "gemv")
        if st is None:
            return None
        e1.record(st)
        e1.synchronize()
        return round(e0.elapsed_time(e1) / n * 1e3, 2)

    for st in streams:
        out["us_by_stream"].append(timed(st))
    out["second_pass_us_by_stream"] = [timed(st) for st in streams]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
