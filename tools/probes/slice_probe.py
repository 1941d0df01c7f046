"""Where config 4's single-GPU launch loses rate (development probe, one MI355X): the tree GEMV
over one 128 GiB A (131072 x 131072) as one launch, as n launches over consecutive row ranges,
and over each row slice of it alone, plus config 2's shape (16384 x 16384) on a 2 GiB buffer of
its own for reference, all in one process, interleaved over rounds. A slice that reads slower
than its neighbours points at where the buffer sits in HBM; every slice as fast as config 2 with
the whole launch slower points at the launch.

    python tools/probes/slice_probe.py [--M 131072] [--K 131072] [--slices 16] [--rounds 3] [--pre-gib 2,32,16]

--pre-gib: device buffers of these sizes allocated (hipMalloc, as the engine does), written and
freed one after another before the big A is allocated — the bench's order (the headline's shard,
then configs 3 and 5) — to see whether the big launch's rate depends on what the device held before.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=131072)
    ap.add_argument("--K", type=int, default=131072)
    ap.add_argument("--slices", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pre-gib", default="")
    args = ap.parse_args()
    M, K, S = args.M, args.K, args.slices
    assert M % S == 0
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    from matvec_mpi_multiplier_amd import multiplier as mm

    for gib in (float(v) for v in args.pre_gib.split(",") if v.strip()):
        rows = int(gib * 2 ** 27) // 16384
        b = mm.DeviceBuffer(rows * 16384)
        check(lib.mvg_synth_fill_device(b.ptr, 16384, rows, 16384, 0, 0, 16384, 7, s), "pre fill")
        check(lib.mvg_stream_sync(s), "sync")
        b.free()
    dA = mm.DeviceBuffer(M * K)  # hipMalloc'd like the engine's shard, not through the caching allocator
    a_ptr = dA.ptr
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(a_ptr, K, M, K, 0, 0, K, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
    A2 = torch.empty(16384 * 16384, dtype=torch.float64, device=dev)
    x2 = torch.empty(16384, dtype=torch.float64, device=dev)
    y2 = torch.empty(16384, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A2.data_ptr(), 16384, 16384, 16384, 0, 0, 16384, 42, s), "fill A2")
    check(lib.mvg_synth_fill_device(x2.data_ptr(), 16384, 1, 16384, 0, 0, 16384, 4242, s), "fill x2")
    torch.cuda.synchronize()
    rows = M // S

    def whole():
        check(lib.mvg_gemv(a_ptr, K, x.data_ptr(), y.data_ptr(), M, K, s), "gemv")

    def split(n):
        r = M // n
        for i in range(n):
            check(lib.mvg_gemv(a_ptr + 8 * i * r * K, K, x.data_ptr(), y.data_ptr() + 8 * i * r, r, K, s), "g")

    def one_slice(i):
        check(lib.mvg_gemv(a_ptr + 8 * i * rows * K, K, x.data_ptr(), y.data_ptr() + 8 * i * rows, rows, K, s),
              "slice")

    def cfg2():
        check(lib.mvg_gemv(A2.data_ptr(), 16384, x2.data_ptr(), y2.data_ptr(), 16384, 16384, s), "cfg2")

    peak = 8e12
    for rnd in range(args.rounds):
        out = {"round": rnd}
        ms = timed(cfg2, 50)
        out["cfg2_us"] = round(ms * 1e3, 2)
        out["cfg2_frac"] = round(8 * (16384 * 16384 + 2 * 16384) / (ms * 1e-3) / peak, 4)
        for n in (1, 8, S):
            ms = timed(whole if n == 1 else (lambda n=n: split(n)), 3)
            out[f"split{n}_ms"] = round(ms, 3)
            out[f"split{n}_frac"] = round(8 * (M * K + K + M) / (ms * 1e-3) / peak, 4)
        fr = []
        for i in range(S):
            ms = timed(lambda i=i: one_slice(i), 5)
            fr.append(round(8 * (rows * K + K + rows) / (ms * 1e-3) / peak, 4))
        out["slice_frac"] = fr
        out["slice_frac_min_max"] = [min(fr), max(fr)]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
