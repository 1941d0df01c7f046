"""Does the first memory a process allocates stream slower for the exact forms? (development
tool) Times the tree GEMV and two exact variants at 16384^2 on an A allocated first in the
process, then on an A allocated after a 40 GiB spacer, then again on the first A.

    python tools/probes/exact_alloc_probe.py [rounds]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def time_all(A, x, y, M, K, s, rounds):
    names = [lib.mvg_gemv_exact_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_variant_count())]
    runs = {"tree": lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)}
    for n in ("hop8_l8_w2_u16", "seqx_r64_t16_b2_g8"):
        v = names.index(n)
        runs[n] = lambda v=v: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)
    out = {k: [] for k in runs}
    for _ in range(rounds):
        for k, fn in runs.items():
            check(fn(), k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            out[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    return {k: round(sorted(v)[len(v) // 2], 1) for k, v in out.items()}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    M = K = 16384
    s = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda:0")
    A1 = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A1.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill")
    print(json.dumps({"A": "first allocation", "us": time_all(A1, x, y, M, K, s, rounds)}), flush=True)
    spacer = torch.empty(40 << 27, dtype=torch.float64, device=dev)  # 40 GiB
    A2 = torch.empty(M * K, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A2.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
    print(json.dumps({"A": "after a 40 GiB spacer", "us": time_all(A2, x, y, M, K, s, rounds)}), flush=True)
    print(json.dumps({"A": "first allocation again", "us": time_all(A1, x, y, M, K, s, rounds)}), flush=True)
    del spacer


if __name__ == "__main__":
    main()
