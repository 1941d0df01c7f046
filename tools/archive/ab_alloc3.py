"""A/B: allocation order and flags vs GEMV speed (development tool).
Allocates several buffers of the same size in sequence (plain hipMalloc and
hipExtMallocWithFlags(hipDeviceMallocContiguous)) and times the same GEMV on each."""
import ctypes as C
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

M, K = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (4194304, 512)
order = sys.argv[3].split(",") if len(sys.argv) > 3 else ["plain", "plain", "contig", "plain"]
nbytes = 8 * (M * K + K + M)
torch.cuda.init()
hip = C.CDLL("libamdhip64.so.7")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
s = torch.cuda.current_stream().cuda_stream
x = torch.empty(K, dtype=torch.float64, device="cuda")
y = torch.empty(M, dtype=torch.float64, device="cuda")
check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill")
bufs = []
for kind in order:
    p = C.c_void_p()
    if kind == "plain":
        rc = hip.hipMalloc(C.byref(p), M * K * 8)
    else:
        rc = hip.hipExtMallocWithFlags(C.byref(p), M * K * 8, 0x4)
    print(f"alloc {kind}: rc {rc} at {hex(p.value or 0)}", flush=True)
    if rc == 0:
        check(lib.mvg_synth_fill_device(p.value, K, M, K, 0, 0, K, 42, s), "fill")
        bufs.append((kind, p.value))
torch.cuda.synchronize()


def ev_time(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for rnd in range(2):
    for i, (kind, a) in enumerate(bufs):
        t = ev_time(lambda: lib.mvg_gemv(a, K, x.data_ptr(), y.data_ptr(), M, K, s))
        print(f"round {rnd} buffer {i} ({kind}): {t*1e3:8.1f} us  {nbytes/t/1e6:7.0f} GB/s", flush=True)
