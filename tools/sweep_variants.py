"""GEMV kernel-variant sweep on one MI355X (development tool, not part of the product).

For each BASELINE shape, times every 16-B variant of mvg_gemv_variant with HIP events on
torch's current stream (interleaved rounds in one process), checks each against rocBLAS
fp64 (torch.mv) to 1e-12, and times the read-only stream microkernel over the same bytes
as the HBM ceiling calibration. Prints one JSON object per (shape, variant).
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

SHAPES = [
    ("cfg2_16384sq", 16384, 16384),
    ("cfg5_shard_524288x512", 524288, 512),
    ("cfg3_g8_strip_65536x8192", 65536, 8192),
    ("cfg4_block_65536x32768", 65536, 32768),
    ("cfg3_g4_strip_65536x16384", 65536, 16384),
    ("mid_1048576x2048", 1048576, 2048),
    ("mid_524288x4096", 524288, 4096),
    ("mid_2097152x1024", 2097152, 1024),
    ("cfg5_full_4194304x512", 4194304, 512),
    ("cfg4_full_131072sq", 131072, 131072),
    ("asym_120x60000", 120, 60000),
    ("asym_1200x60000", 1200, 60000),
    ("wide_64x1048576", 64, 1048576),
    ("wide_1024x131072", 1024, 131072),
    ("mid_2048x65536", 2048, 65536),
    ("mid_4096x16384", 4096, 16384),
    ("mid_8192x16384", 8192, 16384),
    ("mid_4096x32768", 4096, 32768),
    ("mid_1536x32768", 1536, 32768),
    ("cfg3_g1_65536sq", 65536, 65536),
    ("ref_600sq", 600, 600),
    ("ref_1800sq", 1800, 1800),
    ("ref_4200sq", 4200, 4200),
    ("ref_7800sq", 7800, 7800),
    ("ref_10200sq", 10200, 10200),
]


def main():
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    if only:  # literal shapes "MxK" join the named ones
        for n in only:
            if "x" in n and n.replace("x", "").isdigit():
                m, k = (int(v) for v in n.split("x"))
                SHAPES.append((n, m, k))
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    max_elems = max(m * k for n, m, k in SHAPES if not only or n in only)
    buf = torch.empty(max_elems, dtype=torch.float64, device=dev)
    xbuf = torch.empty(max(k for n, m, k in SHAPES if not only or n in only), dtype=torch.float64, device=dev)
    sink = torch.zeros(256 * 16 * 256, dtype=torch.float64, device=dev)
    nvar = lib.mvg_gemv_variant_count()
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    iters = 10
    for name, M, K in SHAPES:
        if only and name not in only:
            continue
        A = buf[: M * K].view(M, K)
        x = xbuf[:K]
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
        check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
        ref = torch.mv(A, x)
        nbytes = 8 * (M * K + K + M)
        results = {}
        prefixes = tuple(p.encode() for p in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["vec", "rowblk"]))
        # a prefix ending in "$" names one variant exactly
        exact = tuple(p[:-1] for p in prefixes if p.endswith(b"$"))
        prefixes = tuple(p for p in prefixes if not p.endswith(b"$"))
        variants = [v for v in range(nvar)
                    if (prefixes and lib.mvg_gemv_variant_name(v).startswith(prefixes))
                    or lib.mvg_gemv_variant_name(v) in exact] + [0]
        y = torch.empty(M, dtype=torch.float64, device=dev)
        for v in variants:
            y.zero_()
            check(lib.mvg_gemv_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s), "gemv")
            rel = ((y - ref).abs() / ref.abs().clamp_min(1e-300)).max().item()
            results[v] = {"rel": rel, "ms": []}
        # stream calibration
        results["stream"] = {"ms": []}
        for _ in range(rounds):
            for v in variants + ["stream"]:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                # warm
                if v == "stream":
                    check(lib.mvg_stream_read(A.data_ptr(), M * K, sink.data_ptr(), s), "stream")
                else:
                    check(lib.mvg_gemv_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s), "g")
                e0.record()
                for _ in range(iters):
                    if v == "stream":
                        lib.mvg_stream_read(A.data_ptr(), M * K, sink.data_ptr(), s)
                    else:
                        lib.mvg_gemv_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)
                e1.record()
                e1.synchronize()
                results[v]["ms"].append(e0.elapsed_time(e1) / iters)
        for v, r in results.items():
            ms = sorted(r["ms"])
            med = ms[len(ms) // 2]
            b = nbytes if v != "stream" else 8 * M * K
            out = {
                "shape": name, "variant": v if v == "stream" else lib.mvg_gemv_variant_name(v).decode(),
                "vid": v, "median_us": round(med * 1e3, 2), "min_us": round(ms[0] * 1e3, 2),
                "GBps_median": round(b / (med * 1e-3) / 1e9, 1), "GBps_best": round(b / (ms[0] * 1e-3) / 1e9, 1),
                "max_rel_vs_rocblas": r.get("rel"),
            }
            print(json.dumps(out), flush=True)
        del ref


if __name__ == "__main__":
    main()
