"""Launch the bit-exact GEMV (and, for comparison, the tree-summed one) on one device-resident
shape, for rocprofv3 counter passes (development tool).

    python tools/exact_probe.py [M] [K] [launches] [exact variant name, "auto" or "panels"]

"tree": the tree-summed kernel alone (no exact launches). "panels": the shard is rewritten once into the engine's column-panel layout
(mvg_panel_relayout, P = mvg_exact_panel_width or 256) and the exact launches run
mvg_gemv_exact_panels on it.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    name = sys.argv[4] if len(sys.argv) > 4 else "auto"
    v = 0
    if name not in ("auto", "panels", "tree"):
        names = [lib.mvg_gemv_exact_variant_name(i).decode() for i in range(lib.mvg_gemv_exact_variant_count())]
        v = names.index(name)
    dA, dx, dy = mm.DeviceBuffer(M * K), mm.DeviceBuffer(K), mm.DeviceBuffer(M)
    check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, None), "fill A")
    check(lib.mvg_synth_fill_device(dx.ptr, K, 1, K, 0, 0, K, 4242, None), "fill x")
    exact = lambda: lib.mvg_gemv_exact_variant(dA.ptr, K, dx.ptr, dy.ptr, M, K, v, None)  # noqa: E731
    if name == "panels":
        P = lib.mvg_exact_panel_width(M, K) or 256
        dAp = mm.DeviceBuffer(M * P * (-(-K // P)))
        check(lib.mvg_panel_relayout(dA.ptr, K, M, K, dAp.ptr, M * P, P, None), "relayout")
        exact = lambda: lib.mvg_gemv_exact_panels(dAp.ptr, M * P, P, dx.ptr, dy.ptr, M, K, 0, None)  # noqa: E731
    for _ in range(n):
        if name != "tree":
            check(exact(), "exact")
        check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, None), "tree")
    check(lib.mvg_stream_sync(None), "sync")
    print(f"exact_probe {M}x{K}: {n} launches of {name} and of the tree kernel")


if __name__ == "__main__":
    main()
