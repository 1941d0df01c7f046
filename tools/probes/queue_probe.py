"""Does the number of HIP streams (hardware queues) a process holds slow the exact GEMV down?
(development tool, one MI355X)

    python tools/probes/queue_probe.py [M] [K] [launches]

Times mvg_gemv (tree) and mvg_gemv_exact on one torch-allocated A, on torch's current stream,
as the process adds HIP streams: none; 1, 2, 3 and 6 more streams that each ran one tiny kernel
(the HIP runtime maps streams onto at most GPU_MAX_HW_QUEUES = 4 hardware queues per process);
then an RCCL communicator and a small engine (its own streams) on top. Three timings per stage,
the stages repeated in reverse at the end. One JSON object per stage.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
        out = {"stage": name, "tree_us": [], "exact_us": []}
        for _ in range(3):
            out["tree_us"].append(t(lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)))
            out["exact_us"].append(t(lambda: lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)))
        print(json.dumps(out), flush=True)

    streams = []

    def add_streams(k):
        for _ in range(k):
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                torch.zeros(1, device="cuda:0").add_(1)
            streams.append(st)
        torch.cuda.synchronize()

    stage("no extra stream")
    for k, total in ((1, 1), (1, 2), (1, 3), (3, 6)):
        add_streams(k)
        stage(f"{total} extra used stream(s)")
    comm = mm.Comm.init_all([0])
    stage("+ RCCL communicator")
    eng = mm.Multiplier("rowwise", 2048, 2048, comm)
    eng.fill_synth()
    eng.multiply()
    eng.sync()
    stage("+ engine (its streams, one multiply)")
    eng.destroy()
    comm.destroy()
    stage("engine and communicator destroyed")


if __name__ == "__main__":
    main()
