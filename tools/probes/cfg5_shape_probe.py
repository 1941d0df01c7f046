"""Config-5 shape probe (development tool): why the one-row-per-wave tree kernel reads a 16 GiB
4,194,304 x 512 A at 0.85-0.91 of peak depending on the box, while its 524,288-row shard reads
0.92. In one process, on the same 16 GiB buffer: the whole launch (auto and a few variants),
eight 524,288-row launches over the same bytes, the same bytes as 16384 x 131072 long rows,
and the read-only stream kernel; then a separate 2 GiB shard. Optional: first allocate and
free a large buffer, as the bench does before config 5 (config 4's 128 GiB).

    python tools/probes/cfg5_shape_probe.py [--pre-gib 128] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def timed(fn, reps):
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


def vid(name):
    for v in range(1, lib.mvg_gemv_variant_count() + 1):
        if lib.mvg_gemv_variant_name(v).decode() == name:
            return v
    raise KeyError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pre-gib", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    if args.pre_gib:
        big = torch.empty(args.pre_gib << 27, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(big.data_ptr(), 131072, big.numel() // 131072, 131072, 0, 0, 131072, 42, s),
              "fill big")
        torch.cuda.synchronize()
        del big
        torch.cuda.empty_cache()
    M, K = 4194304, 512
    A = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(131072, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    sink = torch.zeros(256 * 16 * 256, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), 131072, 1, 131072, 0, 0, 131072, 4242, s), "fill x")
    torch.cuda.synchronize()
    a, xp, yp = A.data_ptr(), x.data_ptr(), y.data_ptr()
    nb = 8 * (M * K + K + M)

    def out(name, t, nbytes=nb):
        print(json.dumps({"case": name, "us": round(t * 1e3, 1), "TBps": round(nbytes / t / 1e9, 3),
                          "addr_GiB": round(a / 2**30, 1)}), flush=True)

    for rnd in range(2):
        out(f"r{rnd} whole auto", timed(lambda: lib.mvg_gemv(a, K, xp, yp, M, K, s), args.reps))
        for name in ("vec_l64_r1_u4_nt1_o5", "vec_l64_r1_u8_nt1_o0", "rowblk_w2_r2_u4", "vec_l64_r2_u8_nt1_o2"):
            v = vid(name)
            out(f"r{rnd} whole {name}", timed(lambda: lib.mvg_gemv_variant(a, K, xp, yp, M, K, v, s), args.reps))

        def eight():
            for p in range(8):
                lib.mvg_gemv(a + p * (M // 8) * K * 8, K, xp, yp + p * (M // 8) * 8, M // 8, K, s)
        out(f"r{rnd} eight 524288-row launches", timed(eight, args.reps))
        out(f"r{rnd} same bytes as 16384x131072",
            timed(lambda: lib.mvg_gemv(a, 131072, xp, yp, 16384, 131072, s), args.reps),
            8 * (16384 * 131072 + 131072 + 16384))
        out(f"r{rnd} stream read 16 GiB",
            timed(lambda: lib.mvg_stream_read(a, M * K, sink.data_ptr(), s), args.reps), 8 * M * K)
    # a separate 2 GiB shard
    B = torch.empty(M // 8 * K, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(B.data_ptr(), K, M // 8, K, 0, 0, K, 42, s), "fill B")
    torch.cuda.synchronize()
    b = B.data_ptr()
    t = timed(lambda: lib.mvg_gemv(b, K, xp, yp, M // 8, K, s), args.reps * 4)
    print(json.dumps({"case": "separate 2 GiB shard auto", "us": round(t * 1e3, 1),
                      "TBps": round(8 * (M // 8 * K + K + M // 8) / t / 1e9, 3),
                      "addr_GiB": round(b / 2**30, 1)}), flush=True)


if __name__ == "__main__":
    main()
