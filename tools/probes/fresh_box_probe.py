"""Does config 2's tree kernel run slower right after a box is handed over? (development probe)

    python tools/probes/fresh_box_probe.py [seconds] [M] [K] [pause]

The first GPU process of a gpurun call: one 2 GiB A, then every `pause` s a burst of 20 back-to-back
mvg_gemv launches timed by one event pair (µs per launch), for `seconds`. Prints one JSON line
per burst (t since start, µs, the device's used VRAM from torch.cuda.mem_get_info and the
current DPM level of each clock domain from sysfs), so a rate that changes over the first minute
shows up beside what the clocks did.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402


def main():
    import torch

    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    pause = float(sys.argv[4]) if len(sys.argv) > 4 else 0.5  # 0: continuous load
    t_start = time.perf_counter()
    torch.cuda.set_device(0)
    dA, dx, dy = mm.DeviceBuffer(M * K), mm.DeviceBuffer(K), mm.DeviceBuffer(M)
    check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, None), "fill A")
    check(lib.mvg_synth_fill_device(dx.ptr, K, 1, K, 0, 0, K, 4242, None), "fill x")
    st = torch.cuda.Stream()
    h = st.cuda_stream
    p = torch.cuda.get_device_properties(0)
    dev_dir = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"

    def clocks():
        """The current DPM level of each clock domain the driver lists (the line marked '*')."""
        out = {}
        for dom in ("sclk", "mclk", "fclk", "socclk"):
            try:
                for line in open(f"{dev_dir}/pp_dpm_{dom}"):
                    if line.rstrip().endswith("*"):
                        out[dom] = line.split(":", 1)[1].strip(" *\n")
            except OSError:
                pass
        return out

    while time.perf_counter() - t_start < secs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, h), "gemv")
        e0.record(st)
        for _ in range(20):
            check(lib.mvg_gemv(dA.ptr, K, dx.ptr, dy.ptr, M, K, h), "gemv")
        e1.record(st)
        e1.synchronize()
        free, total = torch.cuda.mem_get_info(0)
        print(json.dumps({"t": round(time.perf_counter() - t_start, 2), "us": round(e0.elapsed_time(e1) / 20 * 1e3, 2),
                          "vram_used_gib": round((total - free) / 2 ** 30, 1), "clocks": clocks()}), flush=True)
        time.sleep(pause)


if __name__ == "__main__":
    main()
