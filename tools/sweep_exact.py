"""Bit-exact GEMV variants (mvg_gemv_exact_variant) against the tree-summed auto GEMV, one
MI355X (development tool, not part of the product).

    python tools/sweep_exact.py [rounds] [shape,shape,...]

Times every exact variant and the default mvg_gemv on each shape with HIP events (interleaved
rounds, 10 launches per timing), checks that the exact result agrees with the tree-summed one to
1e-12 and is identical run to run, and prints one JSON object per (shape, variant); variants
that refuse a shape's operands (16-B forms on an odd lda) are left out of it.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

SHAPES = [
    ("cfg2_16384sq", 16384, 16384),
    ("cfg5_shard_524288x512", 524288, 512),
    ("cfg3_g8_strip_65536x8192", 65536, 8192),
    ("cfg4_block_65536x32768", 65536, 32768),
    ("cfg5_full_4194304x512", 4194304, 512),
    ("cfg3_g1_65536sq", 65536, 65536),
    ("mid_32768x16384", 32768, 16384),
    ("cfg3_g4_strip_65536x16384", 65536, 16384),
    ("mid_24576x16384", 24576, 16384),
    ("mid_20480x16384", 20480, 16384),
    ("ref_4200sq", 4200, 4200),
    ("ref_10200sq", 10200, 10200),
    ("cfg4_full_131072sq", 131072, 131072),
    ("tall_131072x16384", 131072, 16384),
    ("tall_262144x8192", 262144, 8192),
    ("tall_1048576x2048", 1048576, 2048),
    ("asym_1200x60000", 1200, 60000),
    ("asym_120x60000", 120, 60000),
    ("ref_600sq", 600, 600),
    ("ref_1800sq", 1800, 1800),
    ("mid_4096x16384", 4096, 16384),
    ("mid_8192x16384", 8192, 16384),
    ("mid_4096x32768", 4096, 32768),
    ("mid_2048x65536", 2048, 65536),
    ("mid_8192x8192", 8192, 8192),
    ("mid_12288x12288", 12288, 12288),
    # odd widths (lda = K odd: the 16-B forms refuse, the 8-B ones run): column-split strips of
    # the reference's sizes at P = 8 (4200 / 8 = 525), and odd neighbours of the big shapes
    ("odd_4200x525", 4200, 525),
    ("odd_10200x1275", 10200, 1275),
    ("odd_16384x16383", 16384, 16383),
    ("odd_1200x60001", 1200, 60001),
    ("odd_65536x8191", 65536, 8191),
    ("odd_4096x16383", 4096, 16383),
    # even widths whose rows are 16-B but not 128-B aligned (row stride 131088 / 131104 B)
    ("even_16384x16386", 16384, 16386),
    ("even_16384x16388", 16384, 16388),
    ("even_16384x16400", 16384, 16400),
]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    shapes = [s for s in SHAPES if not only or s[0] in only]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    buf = torch.empty(max(m * k for _, m, k in shapes), dtype=torch.float64, device=dev)
    xbuf = torch.empty(max(k for _, _, k in shapes), dtype=torch.float64, device=dev)
    nvar = lib.mvg_gemv_exact_variant_count()
    for name, M, K in shapes:
        A = buf[: M * K].view(M, K)
        x = xbuf[:K]
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
        check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
        ref = torch.empty(M, dtype=torch.float64, device=dev)
        check(lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), ref.data_ptr(), M, K, s), "gemv")
        nbytes = 8 * (M * K + K + M)
        runs = {"tree": lambda y: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)}
        for v in range(nvar):
            runs[lib.mvg_gemv_exact_variant_name(v).decode()] = (
                lambda y, v=v: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s))
        # calibration: a plain streaming read of A's bytes (every position read once, no chain, no
        # sliding window) — the rate the exact forms' all-rows-at-once access pattern is held to
        sink = torch.empty(1 << 20, dtype=torch.float64, device=dev)
        stream = lambda: lib.mvg_stream_read(A.data_ptr(), M * K, sink.data_ptr(), s)  # noqa: E731
        res = {"stream_read": {"ms": [], "rel": None, "deterministic": None}}
        y = torch.empty(M, dtype=torch.float64, device=dev)
        for key in list(runs):
            if runs[key](y) != 0:  # a 16-B form refusing an odd lda: not a result
                del runs[key]
        for key, fn in runs.items():
            check(fn(y), key)
            y1 = y.clone()
            check(fn(y), key)
            res[key] = {"ms": [], "rel": ((y - ref).abs() / ref.abs().clamp_min(1e-300)).max().item(),
                        "deterministic": bool(torch.equal(y, y1))}
        timed = dict(runs, stream_read=lambda y: stream())
        for _ in range(rounds):
            for key, fn in timed.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                check(fn(y), key)
                e0.record()
                for _ in range(10):
                    fn(y)
                e1.record()
                e1.synchronize()
                res[key]["ms"].append(e0.elapsed_time(e1) / 10)
        for key, r in res.items():
            ms = sorted(r["ms"])
            med = ms[len(ms) // 2]
            print(json.dumps({"shape": name, "M": M, "K": K, "variant": key, "median_us": round(med * 1e3, 2),
                              "min_us": round(ms[0] * 1e3, 2), "GBps_median": round(nbytes / (med * 1e-3) / 1e9, 1),
                              "max_rel_vs_tree": r["rel"], "deterministic": r["deterministic"]}), flush=True)


if __name__ == "__main__":
    main()
