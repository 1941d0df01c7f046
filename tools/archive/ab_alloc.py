"""A/B on one GPU, one process: the same auto GEMV on (a) the engine's own buffers,
(b) torch-allocated buffers, (c) buffers from mvg_malloc — development tool."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

M, K = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (4194304, 512)
alg = sys.argv[3] if len(sys.argv) > 3 else "rowwise"
nbytes = 8 * (M * K + K + M)


def ev_time(fn, iters=20, stream=None):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


comm = mm.Comm.init_all([0])
eng = mm.Multiplier(alg, M, K, comm)
eng.fill_synth()
eng.sync()
s_eng = eng.stream(0)
torch_stream = torch.cuda.ExternalStream(s_eng)
A = torch.empty(M * K, dtype=torch.float64, device="cuda")
x = torch.empty(K, dtype=torch.float64, device="cuda")
y = torch.empty(M, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill")
torch.cuda.synchronize()
for rnd in range(3):
    t_eng = ev_time(lambda: eng.multiply(), stream=torch_stream)
    eng.kernel_timing(True)
    for _ in range(20):
        eng.multiply()
    kt = eng.kernel_ms()
    eng.kernel_timing(False)
    t_torch = ev_time(lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s))
    t_torch_engstream = ev_time(lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s_eng),
                                stream=torch_stream)
    print(f"round {rnd}: engine multiply {t_eng*1e3:.1f} us ({nbytes/t_eng/1e6:.0f} GB/s), engine kernel events "
          f"{kt.avg_ms*1e3:.1f} us, torch buffers {t_torch*1e3:.1f} us ({nbytes/t_torch/1e6:.0f} GB/s), "
          f"torch buffers on engine stream {t_torch_engstream*1e3:.1f} us", flush=True)
