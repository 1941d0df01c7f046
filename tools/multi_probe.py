"""Launch mvg_gemv_multi (several vectors per pass over A, automatic kernel choice) on one
device-resident shape, for rocprofv3 counter passes (development tool).

    python tools/multi_probe.py [M] [K] [launches] [nv<N>]      e.g. 16384 16384 10 nv16

Used as PMC_PROBE=tools/multi_probe.py tools/pmc_passes.sh OUTDIR M K nv8 nv16.
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
    nv = int(sys.argv[4][2:]) if len(sys.argv) > 4 else 8
    dA, dX, dY = mm.DeviceBuffer(M * K), mm.DeviceBuffer(nv * K), mm.DeviceBuffer(nv * M)
    check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, None), "fill A")
    for v in range(nv):
        check(lib.mvg_synth_fill_device(dX.ptr + 8 * K * v, K, 1, K, 0, 0, K, 4242 + v, None), "fill x")
    for _ in range(n):
        check(lib.mvg_gemv_multi(dA.ptr, K, dX.ptr, K, dY.ptr, M, M, K, nv, None), "multi")
    check(lib.mvg_stream_sync(None), "sync")
    name = lib.mvg_gemv_multi_variant_name(lib.mvg_gemv_multi_auto_variant(K, K, M, K, nv)).decode()
    print(f"multi_probe {M}x{K}: {n} launches of {nv} vectors ({name})")


if __name__ == "__main__":
    main()
