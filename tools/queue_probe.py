"""Does anything else the process sets up slow the exact GEMV down? (development tool, one MI355X)

    python tools/queue_probe.py [M] [K] [launches]

Times mvg_gemv (tree) and mvg_gemv_exact on one torch-allocated A, on torch's current stream, at
each stage of a process's life: alone; after an RCCL communicator (mm.Comm.init_all); after an
engine on it (mm.Multiplier: its own streams and buffers); after more HIP streams; after the
engine and the communicator are destroyed. One JSON object per stage.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    s = torch.cuda.current_stream().cuda_stream
    A = torch.empty(M * K, dtype=torch.float64, device="cuda:0")
    x = torch.empty(K, dtype=torch.float64, device="cuda:0")
    y = torch.empty(M, dtype=torch.float64, device="cuda:0")
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill")

    def t(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) / n * 1e3, 2)

    def stage(name):
        out = {"stage": name}
        for _ in range(2):
            out.setdefault("tree_us", []).append(t(lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)))
            out.setdefault("exact_us", []).append(
                t(lambda: lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)))
        print(json.dumps(out), flush=True)

    stage("alone")
    comm = mm.Comm.init_all([0])
    stage("after RCCL communicator (init_all)")
    eng = mm.Multiplier("rowwise", 2048, 2048, comm)
    eng.fill_synth()
    eng.multiply()
    eng.sync()
    stage("after a small engine (its streams, one multiply)")
    extra = [torch.cuda.Stream() for _ in range(6)]
    for st in extra:
        with torch.cuda.stream(st):
            torch.zeros(1, device="cuda:0").add_(1)
    torch.cuda.synchronize()
    stage("after 6 more used torch streams")
    eng.destroy()
    comm.destroy()
    stage("after engine and communicator destroyed")


if __name__ == "__main__":
    main()
