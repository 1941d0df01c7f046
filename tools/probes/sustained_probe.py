"""Per-launch time of the tree GEMV, the row-major exact GEMV and the exact GEMV over column
panels as a function of how many launches run back to back (development tool, one MI355X).

    python tools/probes/sustained_probe.py [M] [K] [rounds]

Short bursts (the variant sweeps: 10 launches per timing) and long runs (the bench: hundreds of
multiplies in a row) can see different rates when a kernel's power draw lowers the sustained
clock; this times bursts of 10, 50 and 200 launches of each kernel, interleaved, on one A.
One JSON object per (kernel, burst).
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
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    A = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
    P = lib.mvg_exact_panel_width(M, K) or 256
    Ap = torch.empty(M * P * (-(-K // P)), dtype=torch.float64, device=dev)
    check(lib.mvg_panel_relayout(A.data_ptr(), K, M, K, Ap.data_ptr(), M * P, P, s), "relayout")
    runs = {
        "tree": lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s),
        "exact_row_major": lambda: lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s),
        "exact_panels": lambda: lib.mvg_gemv_exact_panels(Ap.data_ptr(), M * P, P, x.data_ptr(), y.data_ptr(), M, K,
                                                          0, s),
    }
    nbytes = 8 * (M * K + K + M)
    res = {}
    for _ in range(rounds):
        for n in (10, 50, 200):
            for key, fn in runs.items():
                check(fn(), key)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                e1.synchronize()
                res.setdefault((key, n), []).append(e0.elapsed_time(e1) / n)
    for (key, n), ms in res.items():
        med = sorted(ms)[len(ms) // 2]
        print(json.dumps({"M": M, "K": K, "kernel": key, "burst": n, "median_us": round(med * 1e3, 2),
                          "all_us": [round(v * 1e3, 2) for v in ms], "GBps": round(nbytes / (med * 1e-3) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
