"""Chain-hopping exact GEMV over a column-panel layout of A against the row-major exact dispatch,
the tree kernel and a plain streaming read, one MI355X (development tool, not part of the
product).

    python tools/panel_probe.py [rounds] [shape,shape,...] [P,P,...] [--micro]

For each shape and panel width P: the row-major A is rewritten in panel layout (panel p = columns
[pP, pP + P) of all rows) by mvg_panel_relayout (timed too, `relayout`), every panel variant
(mvg_gemv_exact_panels) runs, its y must equal the row-major exact kernel's y bit for bit, and
each is timed with HIP events (interleaved rounds, 10 launches per timing) beside `tree`
(mvg_gemv), `exact` (mvg_gemv_exact) and `stream_read` on the row-major A. One JSON object per
(shape, P, variant). --micro runs the first prototype (tools/micro/panel_hop.hip ->
tools/micro/libpanel_hop.so, panels written by one device fill per panel) instead.
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

SHAPES = {
    "cfg2_16384sq": (16384, 16384),
    "mid_8192x16384": (8192, 16384),
    "cfg3_g8_strip_65536x8192": (65536, 8192),
    "cfg4_block_65536x32768": (65536, 32768),
    "cfg5_shard_524288x512": (524288, 512),
    "tall_131072x16384": (131072, 16384),
    "cfg3_g1_65536sq": (65536, 65536),
    "cfg3_g4_strip_65536x16384": (65536, 16384),
    "odd_16384x16383": (16384, 16383),
    "even_16384x16386": (16384, 16386),
    "ref_10200sq": (10200, 10200),
    "ref_7800sq": (7800, 7800),
    "mid_6144x2048": (6144, 2048),
    "mid_6144x4096": (6144, 4096),
    "tall_262144x4096": (262144, 4096),
    "tall_1048576x2048": (1048576, 2048),
    "ref_4200sq": (4200, 4200),
    "ref_5400sq": (5400, 5400),
    "mid_4096x16384": (4096, 16384),
    "mid_4096x32768": (4096, 32768),
    "mid_2048x65536": (2048, 65536),
}


def load_micro():
    so = os.path.join(ROOT, "tools", "micro", "libpanel_hop.so")
    m = C.CDLL(so)
    m.panel_hop.restype = C.c_int
    m.panel_hop.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    m.panel_variant_name.restype = C.c_char_p
    return m


def main():
    argv = [a for a in sys.argv[1:] if a != "--micro"]
    use_micro = "--micro" in sys.argv
    rounds = int(argv[0]) if len(argv) > 0 else 5
    names = argv[1].split(",") if len(argv) > 1 else list(SHAPES)
    plist = [int(p) for p in argv[2].split(",")] if len(argv) > 2 else [16, 64, 128, 256, 512, 1024]
    micro = load_micro() if use_micro else None
    nvar = micro.panel_variant_count() if use_micro else lib.mvg_gemv_exact_panel_variant_count()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    big = max(SHAPES[n][0] * SHAPES[n][1] for n in names)
    rowA = torch.empty(big, dtype=torch.float64, device=dev)
    panA = torch.empty(big + max(SHAPES[n][0] for n in names) * max(plist), dtype=torch.float64, device=dev)
    xbuf = torch.empty(max(SHAPES[n][1] for n in names), dtype=torch.float64, device=dev)
    sink = torch.empty(1 << 20, dtype=torch.float64, device=dev)
    for name in names:
        M, K = SHAPES[name]
        A, Ap, x = rowA[: M * K], panA, xbuf[:K]
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
        check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
        want = torch.empty(M, dtype=torch.float64, device=dev)
        check(lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), want.data_ptr(), M, K, s), "exact")
        nbytes = 8 * (M * K + K + M)
        y = torch.empty(M, dtype=torch.float64, device=dev)
        for P in plist:
            if P > K or (use_micro and K % P):
                continue
            relayout = lambda: lib.mvg_panel_relayout(A.data_ptr(), K, M, K, Ap.data_ptr(), M * P, P, s)  # noqa: E731
            if use_micro:
                for p in range(K // P):
                    check(lib.mvg_synth_fill_device(Ap.data_ptr() + 8 * p * M * P, P, M, P, 0, p * P, K, 42, s), "fill")
            else:
                check(relayout(), "relayout")
            # relayout first in each round: it leaves its last writes (the end of the panel copy)
            # in the Infinity Cache, which would flatter the kernel timed right after it
            runs = {} if use_micro else {"relayout": relayout}
            runs |= {
                "tree": lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s),
                "exact": lambda: lib.mvg_gemv_exact(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s),
                "stream_read": lambda: lib.mvg_stream_read(A.data_ptr(), M * K, sink.data_ptr(), s),
            }
            same = {}
            for v in range(nvar):
                if use_micro:
                    fn = (lambda v=v: micro.panel_hop(Ap.data_ptr(), M, K, P, x.data_ptr(), y.data_ptr(), v, s))
                    name_v = micro.panel_variant_name(v).decode()
                else:
                    fn = (lambda v=v: lib.mvg_gemv_exact_panels(Ap.data_ptr(), M * P, P, x.data_ptr(), y.data_ptr(),
                                                                M, K, v, s))
                    name_v = lib.mvg_gemv_exact_panel_variant_name(v).decode()
                y.fill_(-1.0)
                if fn() != 0:
                    continue
                torch.cuda.synchronize()
                key = name_v
                same[key] = bool(torch.equal(y, want))
                runs[key] = fn
            ms = {k: [] for k in runs}
            for _ in range(rounds):
                for key, fn in runs.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    fn()
                    e0.record()
                    for _ in range(10):
                        fn()
                    e1.record()
                    e1.synchronize()
                    ms[key].append(e0.elapsed_time(e1) / 10)
            for key, t in ms.items():
                t = sorted(t)
                med = t[len(t) // 2]
                print(json.dumps({"shape": name, "M": M, "K": K, "P": P, "variant": key,
                                  "median_us": round(med * 1e3, 2), "min_us": round(t[0] * 1e3, 2),
                                  "GBps_median": round(nbytes / (med * 1e-3) / 1e9, 1),
                                  "bit_identical_to_exact": same.get(key)}), flush=True)


if __name__ == "__main__":
    main()
