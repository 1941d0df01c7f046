"""The row-major exact GEMV (and the tree one) on streams of different priority and on several
fresh streams of each, in one process (development tool, one MI355X).

    python tools/probes/priority_probe.py [M] [K] [launches]

tools/probes/queue_probe.py showed the exact kernel's time moving by up to 10 % with the hardware queue
its stream lands on; this asks whether a stream's priority (hipStreamCreateWithPriority through
torch.cuda.Stream(priority=...)) pins it. One JSON object per (priority, stream index).
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
    A = torch.empty(M * K, dtype=torch.float64, device="cuda:0")
    x = torch.empty(K, dtype=torch.float64, device="cuda:0")
    y = torch.empty(M, dtype=torch.float64, device="cuda:0")
    s0 = torch.cuda.current_stream().cuda_stream
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s0), "fill")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s0), "fill")
    torch.cuda.synchronize()
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    streams = []
    for prio in sorted({0, lo, hi}):
        for i in range(3):
            streams.append((prio, i, torch.cuda.Stream(priority=prio)))
    for _ in range(2):
        for prio, i, st in streams:
            s = st.cuda_stream
            out = {"priority": prio, "stream": i}
            for name, fn in (("tree", lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)),
                             ("exact", lambda: lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s))):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(n):
                    fn()
                e1.record(st)
                e1.synchronize()
                out[name + "_us"] = round(e0.elapsed_time(e1) / n * 1e3, 2)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
