"""Zero-copy probe (development tool): can the GEMV read the root's page-locked host A directly
over PCIe faster than the engine's H2D copy + GEMV on the copy?

    python tools/probes/zero_copy_probe.py [--iters 50]

Per size, host-timed medians (stream synchronize at the end of each iteration):
  copy : H2D of A and x (DMA) -> GEMV on the device copy -> D2H of y   (the engine's e2e form)
  zc   : GEMV reading A and x straight from page-locked host memory, y written to device -> D2H
  zc_y : as zc, but the kernel writes y straight into page-locked host memory (one launch)
Every y is compared with the copy form's y (identical kernels, identical order: bit-equal).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def med(fn, iters):
    ts = []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for n in (600, 1800, 4200, 10200, 16384):
        hA = torch.rand(n, n, dtype=torch.float64).pin_memory()
        hx = torch.rand(n, dtype=torch.float64).pin_memory()
        hy = torch.empty(n, dtype=torch.float64).pin_memory()
        dA = torch.empty(n, n, dtype=torch.float64, device=dev)
        dx = torch.empty(n, dtype=torch.float64, device=dev)
        dy = torch.empty(n, dtype=torch.float64, device=dev)

        def copy():
            dA.copy_(hA, non_blocking=True)
            dx.copy_(hx, non_blocking=True)
            check(lib.mvg_gemv(dA.data_ptr(), n, dx.data_ptr(), dy.data_ptr(), n, n, s), "gemv")
            hy.copy_(dy, non_blocking=True)

        def zc():
            check(lib.mvg_gemv(hA.data_ptr(), n, hx.data_ptr(), dy.data_ptr(), n, n, s), "gemv zc")
            hy.copy_(dy, non_blocking=True)

        def zc_y():
            check(lib.mvg_gemv(hA.data_ptr(), n, hx.data_ptr(), hy.data_ptr(), n, n, s), "gemv zc_y")

        out = {"n": n, "A_bytes": 8 * n * n}
        ref = None
        for name, fn in (("copy", copy), ("zc", zc), ("zc_y", zc_y)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            y = hy.clone()
            if ref is None:
                ref = y
            out[name + "_equal"] = bool(torch.equal(y, ref))
            t = med(fn, args.iters)
            out[name + "_ms"] = round(t * 1e3, 4)
            out[name + "_GBps"] = round(8 * n * n / t / 1e9, 2)
        print(json.dumps(out), flush=True)
        del hA, hx, hy, dA, dx, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
