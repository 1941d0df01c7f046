"""Sub-launch probe (development tool): one GEMV launch over a large A against the same product
issued as n launches over consecutive row ranges (n = 1, 2, 4, ... on the same stream). Tests
whether long launches lose rate as the eight XCDs drift apart in the workgroup sequence (a launch
boundary re-aligns them) on the BASELINE config shapes.

    python tools/probes/sublaunch_probe.py [--shapes 4194304x512,65536x65536] [--pre-gib 0]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4194304x512,65536x65536,131072x131072,16384x16384")
    ap.add_argument("--pre-gib", type=int, default=0)
    ap.add_argument("--exact", action="store_true", help="the bit-exact kernels (mvg_gemv_exact)")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="create and use this many more HIP streams first (the engine holds several)")
    ap.add_argument("--nv", type=int, default=1, help="vectors per pass (mvg_gemv_multi) when > 1")
    ap.add_argument("--splits", default="1,2,4,8,16,32,64")
    ap.add_argument("--piece-rows", default="", help="instead of --splits: launches of at most this many rows "
                    "(comma list; the last launch takes the remainder)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    gemv = lib.mvg_gemv_exact if args.exact else lib.mvg_gemv
    extra = [torch.cuda.Stream() for _ in range(args.extra_streams)]
    for st in extra:
        with torch.cuda.stream(st):
            torch.ones(1, device=dev).add_(1)
    torch.cuda.synchronize()
    if args.pre_gib:
        big = torch.empty(args.pre_gib << 27, dtype=torch.float64, device=dev)
        big.zero_()
        torch.cuda.synchronize()
        del big
        torch.cuda.empty_cache()
    for shape in args.shapes.split(","):
        M, K = (int(v) for v in shape.split("x"))
        A = torch.empty(M * K, dtype=torch.float64, device=dev)
        nv = args.nv
        x = torch.empty(K * nv, dtype=torch.float64, device=dev)
        y = torch.empty(M * nv, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
        check(lib.mvg_synth_fill_device(x.data_ptr(), K, nv, K, 0, 0, K, 4242, s), "fill x")
        torch.cuda.synchronize()
        a, xp, yp = A.data_ptr(), x.data_ptr(), y.data_ptr()
        nb = 8 * (M * K + nv * (K + M))
        reps = max(2, int(2e9 / nb * 10)) if nb < 2e10 else 2
        ref = None
        for rnd in range(2):
            cases = ([(M // n, n) for n in (int(v) for v in args.splits.split(",")) if M % n == 0 and (M // n) % 2 == 0]
                     if not args.piece_rows else
                     [(int(v), -(-M // int(v))) for v in args.piece_rows.split(",")])
            for rows, n in cases:
                def run():
                    for r0 in range(0, M, rows):
                        r = min(rows, M - r0)
                        if nv > 1:
                            lib.mvg_gemv_multi(a + r0 * K * 8, K, xp, K, yp + r0 * 8, M, r, K, nv, s)
                        else:
                            gemv(a + r0 * K * 8, K, xp, yp + r0 * 8, r, K, s)
                t = timed(run, reps)
                if ref is None:
                    ref = y.clone()
                same = bool(torch.equal(ref, y))
                print(json.dumps({"shape": shape, "exact": args.exact, "nv": nv, "round": rnd, "launches": n, "rows_per_launch": rows, "GiB_per_launch": round(8 * rows * K / 2**30, 3),
                                  "us": round(t * 1e3, 1), "TBps": round(nb / t / 1e9, 3), "y_identical": same,
                                  "addr_GiB": round(a / 2**30, 1)}), flush=True)
        del A, x, y, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
