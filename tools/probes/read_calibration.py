"""Read-rate calibration on one MI355X (development tool, not part of the product): the tree GEMV
(mvg_gemv) beside read-only kernels over the same bytes — an address-order grid-stride sweep
(tools/micro/seq_read.hip, several grid sizes and load depths), per-wave contiguous ranges, and
the product's mvg_stream_read — to place the GEMV against the best read rate the chip gives.

    python tools/probes/read_calibration.py [rounds] [M,K ...]

One JSON object per (shape, kernel): median / min microseconds over interleaved rounds of 10
launches, and GB/s of the A bytes (reads of x and writes of y excluded for the read kernels;
the GEMV's GB/s uses its algorithmic bytes 8(MK + K + M)).
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(16384, 16384), (65536, 32768)]
    micro = C.CDLL(os.path.join(ROOT, "tools", "micro", "libseq_read.so"))
    micro.read_kernel.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    big = max(m * k for m, k in shapes)
    A = torch.empty(big, dtype=torch.float64, device=dev)
    xb = torch.empty(max(k for _, k in shapes), dtype=torch.float64, device=dev)
    y = torch.empty(max(m for m, _ in shapes), dtype=torch.float64, device=dev)
    sink = torch.empty(1 << 16, dtype=torch.float64, device=dev)
    for M, K in shapes:
        n = M * K
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
        check(lib.mvg_synth_fill_device(xb.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
        runs = {"gemv_tree": lambda: lib.mvg_gemv(A.data_ptr(), K, xb.data_ptr(), y.data_ptr(), M, K, s),
                "stream_read": lambda: lib.mvg_stream_read(A.data_ptr(), n, sink.data_ptr(), s)}
        for blocks in (1024, 2048, 4096, 8192):
            for unr in (4, 8, 16):
                runs[f"seq_b{blocks}_u{unr}"] = (lambda b=blocks, u=unr:
                                                 micro.read_kernel(0, u, b, A.data_ptr(), n, sink.data_ptr(), s))
        for blocks in (1024, 4096):
            runs[f"range_b{blocks}_u8"] = (lambda b=blocks: micro.read_kernel(1, 8, b, A.data_ptr(), n, sink.data_ptr(), s))
        for key, fn in runs.items():
            assert fn() == 0, key
        ms = {k: [] for k in runs}
        for _ in range(rounds):
            for key, fn in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn()
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                e1.synchronize()
                ms[key].append(e0.elapsed_time(e1) / 10)
        for key, t in ms.items():
            t = sorted(t)
            med = t[len(t) // 2]
            nbytes = 8 * (n + K + M) if key == "gemv_tree" else 8 * n
            print(json.dumps({"M": M, "K": K, "kernel": key, "median_us": round(med * 1e3, 2),
                              "min_us": round(t[0] * 1e3, 2), "GBps_median": round(nbytes / (med * 1e-3) / 1e9, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
