"""Does an idle gap before a burst change the burst's kernel times? (development probe)

    python tools/probes/idle_gap_probe.py [rounds] [M] [K]

The bench's headline runs K = 20 launches after a settle, a host-side collection and W warm-up
steps; its kernels average ~297 us while the settle's own back-to-back bursts read ~294. This
probe loads the GPU continuously for 1.5 s, then per round and per gap (interleaved): 0.3 s of
continuous load, the gap (idle: a sleep, or one gc.collect() as the bench runs), then 20
mvg_gemv launches with an event before each launch and after the last, so every launch's own
duration is measured. One JSON line per (round, gap): the gap's length, the 20 per-launch us,
their mean, and the shader clock's DPM level before and after the burst.
"""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    import torch

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    torch.cuda.set_device(0)
    dA, dx, dy = mm.DeviceBuffer(M * K), mm.DeviceBuffer(K), mm.DeviceBuffer(M)
    check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, None), "fill A")
    check(lib.mvg_synth_fill_device(dx.ptr, K, 1, K, 0, 0, K, 4242, None), "fill x")
    st = torch.cuda.Stream()
    h = st.cuda_stream
    p = torch.cuda.get_device_properties(0)
    dev_dir = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"

    def sclk():
        try:
            for line in open(f"{dev_dir}/pp_dpm_sclk"):
                if line.rstrip().endswith("*"):
                    return line.split(":", 1)[1].strip(" *\n")
        except OSError:
            pass
        return None

    def gemv():
        check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, h), "gemv")

    def load(seconds):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(20):
                gemv()
            st.synchronize()

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    ev[0].record(st)
    ev[1].record(st)
    st.synchronize()  # the events' first use outside any burst
    load(1.5)
    gaps = ["none", 0.001, 0.01, "gc", 0.05, 0.2]
    for r in range(rounds):
        for gap in gaps:
            load(0.3)
            c0 = sclk()
            t0 = time.perf_counter()
            if gap == "gc":
                gc.collect()
            elif gap != "none":
                time.sleep(gap)
            idle = time.perf_counter() - t0
            for i in range(20):
                ev[i].record(st)
                gemv()
            ev[20].record(st)
            ev[20].synchronize()
            us = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(20)]
            print(json.dumps({"round": r, "gap": gap, "idle_ms": round(idle * 1e3, 2), "mean_us": round(sum(us) / 20, 2),
                              "first5_us": round(sum(us[:5]) / 5, 1), "last5_us": round(sum(us[-5:]) / 5, 1),
                              "sclk_before": c0, "sclk_after": sclk(), "us": us}), flush=True)


if __name__ == "__main__":
    main()
