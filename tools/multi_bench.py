"""mvg_gemv_multi (several x per pass over A): every kernel variant against nv separate mvg_gemv
calls (development tool). Prints one JSON line per (shape, nv, variant): time per call, the A-stream rate (8*M*K bytes / time) and the max relative error against rocBLAS (torch).

    python tools/multi_bench.py [MxK,...|all] [variant-name-prefix,...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402

SHAPES = [(16384, 16384), (65536, 8192), (4194304, 512), (1048576, 2048), (524288, 4096), (2097152, 1024),
          (8192, 65536), (4200, 4200)]


def timeit(fn, reps=10, rounds=5):
    times = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1) / reps)
    return sorted(times)[rounds // 2]


def main():
    only = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] != "all" else None
    vfilter = sys.argv[2].split(",") if len(sys.argv) > 2 else None  # variant name prefixes
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    nvar = lib.mvg_gemv_multi_variant_count()
    for M, K in [tuple(map(int, o.split("x"))) for o in only] if only else SHAPES:
        A = torch.empty(M, K, dtype=torch.float64, device=dev)
        check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill")
        X = torch.rand(16, K, dtype=torch.float64, device=dev)
        Y = torch.empty(16, M, dtype=torch.float64, device=dev)
        ref = X @ A.T  # rocBLAS
        for nv in (2, 4, 8, 16):
            cands = [("separate", None)] + [(lib.mvg_gemv_multi_variant_name(v).decode(), v) for v in range(nvar)]
            for name, v in cands:
                if vfilter and v is not None and not any(name.startswith(f) for f in vfilter):
                    continue
                if v is None:
                    def fn():
                        for j in range(nv):
                            check(lib.mvg_gemv(A.data_ptr(), K, X[j].data_ptr(), Y[j].data_ptr(), M, K, s), "gemv")
                else:
                    def fn(v=v):
                        check(lib.mvg_gemv_multi_variant(A.data_ptr(), K, X.data_ptr(), K, Y.data_ptr(), M, M, K,
                                                         nv, v, s), "multi")
                Y.zero_()
                fn()
                torch.cuda.synchronize()
                err = ((Y[:nv] - ref[:nv]).abs() / ref[:nv].abs()).max().item()
                ms = timeit(fn)
                print(json.dumps({"M": M, "K": K, "nv": nv, "variant": name, "ms": round(ms, 4),
                                  "A_GBps": round(8 * M * K / (ms * 1e-3) / 1e9, 1), "max_rel": err}), flush=True)
        del A, X, Y, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
