"""Placement probe (development tool): the same GEMV variants on many freshly allocated buffers of
one shape in one process, to find buffers whose placement reads slower and which kernel orders
are immune to it. `pieces<n>` = the dispatch's kernel as n launches over consecutive row ranges;
`stream` = the read-only stream kernel over A's bytes; `exact` = the dispatch's bit-exact kernel.

    python tools/probes/placement_probe.py [--shape 16384x16384] [--buffers 12]
        [--variants auto,rowblk_w4_r2_u8_xcd,pieces2,stream]
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
    ap.add_argument("--shape", default="16384x16384")
    ap.add_argument("--buffers", type=int, default=12)
    ap.add_argument("--variants", default="auto,rowblk_w4_r2_u8_xcd,rowblk_w4_r2_u8_xq64,rowblk_w8_r2_u4,"
                                         "vec_l64_r2_u4_nt1_o7,pieces2,stream")
    args = ap.parse_args()
    M, K = (int(v) for v in args.shape.split("x"))
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    names = {lib.mvg_gemv_variant_name(v).decode(): v for v in range(lib.mvg_gemv_variant_count())}
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    sink = torch.zeros(1 << 20, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
    bufs = []
    for _ in range(args.buffers):
        A = torch.empty(M * K, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
        bufs.append(A)
    torch.cuda.synchronize()
    nb = 8 * (M * K + K + M)
    reps = max(3, int(4e9 / nb * 10))
    xp, yp = x.data_ptr(), y.data_ptr()
    for rnd in range(2):
        for b, A in enumerate(bufs):
            a = A.data_ptr()
            out = {"round": rnd, "buffer": b, "addr_GiB": round(a / 2**30, 2)}
            for name in args.variants.split(","):
                if name == "exact":
                    fn = (lambda: lib.mvg_gemv_exact(a, K, xp, yp, M, K, s))
                elif name == "stream":
                    fn = (lambda: lib.mvg_stream_read(a, M * K, sink.data_ptr(), s))
                elif name.startswith("pieces"):
                    n = int(name[6:])
                    rows = (M // n + 1) // 2 * 2

                    def fn(n=n, rows=rows):
                        for r0 in range(0, M, rows):
                            lib.mvg_gemv(a + r0 * K * 8, K, xp, yp + r0 * 8, min(rows, M - r0), K, s)
                else:
                    v = 0 if name == "auto" else names[name]
                    fn = (lambda v=v: lib.mvg_gemv_variant(a, K, xp, yp, M, K, v, s))
                out[name] = round(timed(fn, reps) * 1e3, 1)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
