"""H2D bandwidth from pinned host memory first-touched on each NUMA node (development tool).

Prints the GPU's PCI NUMA node, then for every NUMA node: the H2D rate of a 2 GiB buffer whose
pages were first touched by threads bound to that node's CPUs."""
import ctypes as C
import glob
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd._lib import lib, check  # noqa: E402


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += range(int(a), int(b) + 1)
        elif part:
            out.append(int(part))
    return out


def main():
    dev = torch.device("cuda:0")
    bus = torch.cuda.get_device_properties(0)
    pci = getattr(bus, "pci_bus_id", None)
    nodes = sorted(int(p.split("node")[-1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
    gpu_nodes = {}
    for d in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            gpu_nodes[d] = open(d).read().strip()
        except OSError:
            pass
    print(json.dumps({"nodes": nodes, "gpu_numa": gpu_nodes, "pci_bus_id": pci,
                      "allowed_cpus": len(os.sched_getaffinity(0))}), flush=True)
    n = (2 << 30) // 8
    d = torch.empty(n, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    keep = os.sched_getaffinity(0)
    for node in nodes:
        cpus = set(cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read())) & keep
        if not cpus:
            continue
        os.sched_setaffinity(0, cpus)
        a = np.empty(n, dtype=np.float64)
        check(lib.mvg_synth_fill_host(a.ctypes.data, n // 1024, 1024, n // 1024, 0, 0, n // 1024, 1), "fill")  # first touch
        os.sched_setaffinity(0, keep)
        check(lib.mvg_host_register(a.ctypes.data, a.nbytes), "register")
        rates = []
        for _ in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            check(lib.mvg_memcpy_h2d(d.data_ptr(), a.ctypes.data, a.nbytes, s), "h2d")
            torch.cuda.synchronize()
            rates.append(a.nbytes / (time.perf_counter() - t) / 1e9)
        lib.mvg_host_unregister(a.ctypes.data)
        print(json.dumps({"node": node, "cpus": len(cpus), "h2d_GBps": [round(r, 1) for r in rates]}), flush=True)
        del a


if __name__ == "__main__":
    main()
