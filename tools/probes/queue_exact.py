"""Does the hardware queue a stream lands on change a kernel's speed? (development tool, one MI355X)

    python tools/probes/queue_exact.py [M] [K] [launches] [streams]

HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues round robin. The same kernels — the
tree GEMV and the row-major exact GEMV, whose 2048 waves all stay resident for the whole launch —
are timed on the default stream and on `streams` fresh streams of one process, interleaved twice,
each timing `launches` back-to-back launches after 0.1 s of load. One JSON line per (stream, kernel).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    ns = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    dev = torch.device("cuda:0")
    A = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    s0 = torch.cuda.current_stream()
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s0.cuda_stream), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s0.cuda_stream), "fill x")
    streams = [("default", s0)] + [(f"stream{i}", torch.cuda.Stream(device=dev)) for i in range(ns)]
    names = [lib.mvg_gemv_exact_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_variant_count())]
    hop = names.index("hop8_l8_w2_u16")
    kernels = {
        "tree": lambda s: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s),
        "exact_hop8": lambda s: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, hop, s),
    }
    res = {}
    for _ in range(2):
        for sname, st in streams:
            h = st.cuda_stream
            for kname, f in kernels.items():
                torch.cuda.synchronize()
                for _ in range(int(0.1 / 300e-6)):
                    kernels["tree"](h)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
                with torch.cuda.stream(st):
                    for a, b in ev:
                        a.record(st)
                        f(h)
                        b.record(st)
                torch.cuda.synchronize()
                us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
                res.setdefault((sname, kname), []).append(round(us[n // 2], 2))
    for (sname, kname), v in res.items():
        print(json.dumps({"M": M, "K": K, "stream": sname, "kernel": kname, "median_us": v}), flush=True)


if __name__ == "__main__":
    main()
