"""Exact GEMV forms under sustained load (development tool, one MI355X): does a form's speed
hold when the chip has been streaming for a while, as in the bench's exact sections?

    python tools/probes/sustained_exact.py [M] [K] [launches]

For each form (the tree GEMV, the row-major exact variants, the panel form): a 100 ms burst of
tree launches to heat the chip, then `launches` back-to-back launches of the form, each bracketed
by its own HIP events; prints one JSON line per form with the median / p10 / p90 duration, the
first and last tenth's medians (the drift) and, when rocm-smi answers, the GPU's clock, power
and temperature after the run. Two passes in opposite orders.
"""
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

FORMS = ["tree", "hop8_l8_w2_u16", "hop8_l8_w2_u24", "seqx_r64_t16_b2_g8", "seqx_r32_t64_b2_g8",
         "seqx_r64_t32_b2_g8", "panels"]


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showtemp", "--json"],
                           capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        keep = {k: v for k, v in card.items() if any(s in k.lower() for s in ("sclk", "power", "junction", "memory"))}
        return keep
    except Exception as exc:  # informative only
        return {"error": str(exc)[:80]}


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    A = torch.empty(M * K, dtype=torch.float64, device=dev)
    x = torch.empty(K, dtype=torch.float64, device=dev)
    y = torch.empty(M, dtype=torch.float64, device=dev)
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
    names = [lib.mvg_gemv_exact_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_variant_count())]
    P = 256
    Ap = torch.empty(M * P * (-(-K // P)), dtype=torch.float64, device=dev)
    check(lib.mvg_panel_relayout(A.data_ptr(), K, M, K, Ap.data_ptr(), M * P, P, s), "relayout")

    def fn(form):
        if form == "tree":
            return lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)
        if form == "panels":
            return lambda: lib.mvg_gemv_exact_panels(Ap.data_ptr(), M * P, P, x.data_ptr(), y.data_ptr(), M, K, 0, s)
        v = names.index(form)
        return lambda: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)

    heat = fn("tree")
    for order in (FORMS, FORMS[::-1]):
        for form in order:
            f = fn(form)
            if f() != 0:
                continue
            torch.cuda.synchronize()
            for _ in range(max(1, int(0.1 / 300e-6))):
                heat()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
            for a, b in ev:
                a.record()
                f()
                b.record()
            torch.cuda.synchronize()
            us = [a.elapsed_time(b) * 1e3 for a, b in ev]
            srt = sorted(us)
            tenth = max(1, n // 10)
            print(json.dumps({"M": M, "K": K, "form": form, "launches": n, "median_us": round(srt[n // 2], 2),
                              "p10_us": round(srt[n // 10], 2), "p90_us": round(srt[9 * n // 10], 2),
                              "first_tenth_us": round(sorted(us[:tenth])[tenth // 2], 2),
                              "last_tenth_us": round(sorted(us[-tenth:])[tenth // 2], 2),
                              "TBps_median": round(8 * (M * K + K + M) / (srt[n // 2] * 1e-6) / 1e12, 3),
                              "smi_after": smi()}), flush=True)


if __name__ == "__main__":
    main()
