"""A/B: which buffer's allocation (A, x or y; hipMalloc via the library vs torch's caching
allocator) changes the GEMV's speed — development tool."""
import ctypes as C
import itertools
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

M, K = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (4194304, 512)
nbytes = 8 * (M * K + K + M)
s = torch.cuda.current_stream().cuda_stream


def mvg_alloc(n):
    p = C.c_void_p()
    check(lib.mvg_malloc(C.byref(p), n * 8), "malloc")
    return p.value


bufs = {}
for name, n in (("A", M * K), ("x", K), ("y", M)):
    t = torch.empty(n, dtype=torch.float64, device="cuda")
    bufs[(name, "torch")] = (t.data_ptr(), t)
    bufs[(name, "mvg")] = (mvg_alloc(n), None)
for kind in ("torch", "mvg"):
    check(lib.mvg_synth_fill_device(bufs[("A", kind)][0], K, M, K, 0, 0, K, 42, s), "fill")
    check(lib.mvg_synth_fill_device(bufs[("x", kind)][0], K, 1, K, 0, 0, K, 4242, s), "fill")
torch.cuda.synchronize()
print("addresses:", {f"{k[0]}/{k[1]}": hex(v[0]) for k, v in bufs.items()}, flush=True)


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
    for ka, kx, ky in itertools.product(("torch", "mvg"), repeat=3):
        a, x, y = bufs[("A", ka)][0], bufs[("x", kx)][0], bufs[("y", ky)][0]
        t = ev_time(lambda: lib.mvg_gemv(a, K, x, y, M, K, s))
        print(f"round {rnd} A={ka:5s} x={kx:5s} y={ky:5s}: {t*1e3:8.1f} us  {nbytes/t/1e6:7.0f} GB/s", flush=True)
