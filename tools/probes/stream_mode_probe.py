"""Is config 5's slow mode a property of the process or of the HIP stream (hardware queue) a long
launch goes to? (development tool). One 16 GiB A; the one-row-per-wave kernel as ONE launch
(`vec_l64_r1_u8_nt1_o0`, which the 1 GiB launch rule does not split; same two rates as the
dispatch's form) on torch's default stream and on `--streams` more streams of the process, in
turn, twice; then the dispatch's split form on each.

    python tools/probes/stream_mode_probe.py [--streams 6]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def timed(fn, stream, reps=10):
    ts = []
    with torch.cuda.stream(stream):
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=6)
    ap.add_argument("--buffers", type=int, default=1, help="more 16 GiB buffers, each timed on the default stream")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M, K = 4194304, 512
    A = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    s0 = torch.cuda.current_stream()
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s0.cuda_stream), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s0.cuda_stream), "fill x")
    torch.cuda.synchronize()
    one = [v for v in range(1, lib.mvg_gemv_variant_count() + 1)
           if lib.mvg_gemv_variant_name(v).decode() == "vec_l64_r1_u8_nt1_o0"][0]
    streams = [s0] + [torch.cuda.Stream() for _ in range(args.streams)]
    a, xp, yp = A.data_ptr(), x.data_ptr(), y.data_ptr()
    for rnd in range(2):
        for i, st in enumerate(streams):
            h = st.cuda_stream
            t1 = timed(lambda: lib.mvg_gemv_variant(a, K, xp, yp, M, K, one, h), st)
            ta = timed(lambda: lib.mvg_gemv(a, K, xp, yp, M, K, h), st)
            print(json.dumps({"round": rnd, "stream": i, "one_launch_us": round(t1 * 1e3, 1),
                              "dispatch_1GiB_launches_us": round(ta * 1e3, 1)}), flush=True)
    # the same on further buffers (placement) in this process, default stream
    bufs = [A]
    for b in range(1, args.buffers):
        B = torch.empty(M * K, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(B.data_ptr(), K, M, K, 0, 0, K, 42, s0.cuda_stream), "fill B")
        bufs.append(B)
    torch.cuda.synchronize()
    for rnd in range(2):
        for b, B in enumerate(bufs):
            p, h = B.data_ptr(), s0.cuda_stream
            t1 = timed(lambda: lib.mvg_gemv_variant(p, K, xp, yp, M, K, one, h), s0)
            ta = timed(lambda: lib.mvg_gemv(p, K, xp, yp, M, K, h), s0)
            print(json.dumps({"round": rnd, "buffer": b, "addr_GiB": round(p / 2**30, 1),
                              "one_launch_us": round(t1 * 1e3, 1), "dispatch_1GiB_launches_us": round(ta * 1e3, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
