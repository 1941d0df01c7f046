"""Does a large hipFree slow the kernels that run right after it (development probe, one MI355X)?

The kernel driver may clear freed VRAM in the background; that clearing would share HBM with
whatever runs next. The probe allocates a buffer of --gib GiB (hipMalloc, as the engine does),
writes it, frees it, and then, for --seconds, times config 2's GEMV (16384 x 16384, a 2 GiB
buffer held throughout) in bursts of --burst launches while it polls hipMemGetInfo's free
memory and the device's sysfs mem_info_vram_used. One JSON line per burst: seconds since the
free, microseconds per launch, free and used GiB. A baseline phase before the allocation gives
the undisturbed time.

    python tools/probes/vram_clear_probe.py [--gib 128] [--seconds 30] [--burst 20]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def sysfs_used(dev=0):
    """Bytes of VRAM in use on GPU `dev` as its driver counts them (every process; sysfs of the
    device's own PCI address — the host's other GPUs are listed too), None when unreadable."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        return int(open(f"/sys/bus/pci/devices/{bdf}/mem_info_vram_used").read().strip())
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=128)
    ap.add_argument("--seconds", type=float, default=30)
    ap.add_argument("--burst", type=int, default=20)
    args = ap.parse_args()
    s = torch.cuda.current_stream().cuda_stream
    N = 16384
    A = mm.DeviceBuffer(N * N)
    x, y = mm.DeviceBuffer(N), mm.DeviceBuffer(N)
    check(lib.mvg_synth_fill_device(A.ptr, N, N, N, 0, 0, N, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.ptr, N, 1, N, 0, 0, N, 4242, s), "fill x")
    check(lib.mvg_stream_sync(s), "sync")

    def burst():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.burst):
            lib.mvg_gemv(A.ptr, N, x.ptr, y.ptr, N, N, s)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / args.burst * 1e3

    last = [0.0]

    def sample(phase, t0):
        us = burst()
        if time.perf_counter() - last[0] < 0.05:  # one line per 50 ms
            return
        last[0] = time.perf_counter()
        free, total = torch.cuda.mem_get_info(0)
        used = sysfs_used()
        print(json.dumps({"phase": phase, "t": round(time.perf_counter() - t0, 3), "us": round(us, 2),
                          "free_gib": round(free / 2 ** 30, 2), "total_gib": round(total / 2 ** 30, 2),
                          "sysfs_used_gib": round(used / 2 ** 30, 2) if used is not None else None}), flush=True)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        sample("baseline", t0)
    rows = int(args.gib * 2 ** 27) // N
    big = mm.DeviceBuffer(rows * N)
    check(lib.mvg_synth_fill_device(big.ptr, N, rows, N, 0, 0, N, 7, s), "fill big")
    check(lib.mvg_stream_sync(s), "sync")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        sample("big_held", t0)
    big.free()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        sample("after_free", t0)
    for b in (A, x, y):
        b.free()


if __name__ == "__main__":
    main()
