"""The root's host matrix in shared memory, for one process per GPU on one node.

The reference's drivers keep A on the root and scatter it (MPI_Scatter / Pack + Send; on one
host MPICH moves it through shared memory). The MI355X-node form: rank 0 places A in a POSIX
shared-memory segment, every rank maps it, and each GPU pulls its own shard over its own PCIe
link (Multiplier.distribute_shared). Collective over the default torch.distributed group.

Page placement is NUMA-aware: the segment is created empty and every rank first-touches (fills)
its own share of the rows with its threads bound to the CPUs of its GPU's NUMA node, so on a
two-socket MI355X node each GPU's row shard lands in the DRAM of the socket its PCIe link hangs
off — the placement an MPI-3 shared window with per-rank segments gives, instead of the whole
matrix on one socket feeding eight GPUs across the inter-socket link.
"""
from __future__ import annotations

import os
import time
from multiprocessing import resource_tracker, shared_memory

import numpy as np

from ._lib import check, lib

SHM_DIR = "/dev/shm"


def _cpulist(text: str) -> set[int]:
    out: set[int] = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


def device_numa_cpus(device: int) -> set[int] | None:
    """The CPUs (within this process's allowed set) of the NUMA node GPU `device` is attached
    to, from its PCI address in sysfs; None when unknown (no NUMA info, one node, no overlap)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        if node < 0:
            return None
        cpus = _cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()) & os.sched_getaffinity(0)
        return cpus or None
    except Exception:
        return None


def cpu_quota() -> int:
    """The CPUs this process may run on: its affinity mask, capped by its cgroup's CPU quota
    (cpu.max), at most 64 — the library's own host thread count without $MVG_THREADS
    (csrc/host.cpp host_thread_count)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(period) > 0:
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, min(64, n))


def fill_threads(local_ranks: int) -> int:
    """Fill threads per rank when `local_ranks` ranks share this node's CPUs: the CPU quota
    split evenly, at least 1. Without the split every rank starts the whole quota's worth of
    threads, and N ranks oversubscribe the quota N times."""
    return max(1, cpu_quota() // max(1, local_ranks))


def shm_free_bytes() -> int:
    try:
        st = os.statvfs(SHM_DIR)
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


class SharedHostMatrix:
    """R x C fp64 matrix in a shared-memory segment created by rank 0 and mapped by all ranks.

    `create(R, C, seed, tag)` is collective; every rank gets `.array` (the same bytes), or the
    call returns None on every rank when the segment does not fit (decided collectively)."""

    def __init__(self, shm: shared_memory.SharedMemory, shape: tuple[int, int], owner: bool):
        self.shm = shm
        self.owner = owner
        self.array = np.ndarray(shape, dtype=np.float64, buffer=shm.buf)
        self.timing: dict = {}  # this rank's share of the setup: rows, threads, fill seconds

    @classmethod
    def create(cls, R: int, C: int, seed: int, tag: str, device: str = "cpu", margin: int = 1 << 30,
               threads: int | None = None):
        """`threads`: the fill threads of this rank (default: the library's host thread count,
        $MVG_THREADS or the process's CPU quota). Ranks sharing one node's CPUs should split them
        (fill_threads())."""
        import torch
        import torch.distributed as dist

        nbytes = max(R * C * 8, 8)
        ok = torch.tensor([1 if shm_free_bytes() > nbytes + margin else 0], device=device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok[0]):
            return None
        name = f"mvg_{tag}"
        me = None
        if dist.get_rank() == 0:
            try:
                shm = shared_memory.SharedMemory(name=name, create=True, size=nbytes)
            except FileExistsError:  # left behind by a killed run with the same tag: replace it
                stale = shared_memory.SharedMemory(name=name)
                stale.close()
                stale.unlink()
                shm = shared_memory.SharedMemory(name=name, create=True, size=nbytes)
            me = cls(shm, (R, C), owner=True)
        dist.barrier()
        if dist.get_rank() != 0:
            shm = shared_memory.SharedMemory(name=name)
            # only the creator owns (and unlinks) the segment; Python 3.10 registers attachers too
            resource_tracker.unregister(shm._name, "shared_memory")
            me = cls(shm, (R, C), owner=False)
        # first touch: rank r fills rows [r*R/n, (r+1)*R/n) from its GPU's NUMA node
        n, r = dist.get_world_size(), dist.get_rank()
        r0, r1 = R * r // n, R * (r + 1) // n
        t0 = time.perf_counter()
        if r1 > r0 and C:
            cpus = device_numa_cpus(int(str(device).split(":")[1])) if str(device).startswith("cuda:") else None
            keep = os.sched_getaffinity(0)
            had = os.environ.get("MVG_THREADS")
            if cpus:
                os.sched_setaffinity(0, cpus)
            if threads:
                os.environ["MVG_THREADS"] = str(threads)
            try:
                check(lib.mvg_synth_fill_host(me.array[r0:].ctypes.data, C, r1 - r0, C, r0, 0, C, seed),
                      "mvg_synth_fill_host")
            finally:
                if cpus:
                    os.sched_setaffinity(0, keep)
                if threads:
                    if had is None:
                        os.environ.pop("MVG_THREADS", None)
                    else:
                        os.environ["MVG_THREADS"] = had
        me.timing = {"rows": r1 - r0, "threads": threads, "fill_s": round(time.perf_counter() - t0, 3)}
        dist.barrier()
        me.timing["fill_wait_s"] = round(time.perf_counter() - t0, 3)  # until every rank's share is in
        return me

    def close(self) -> None:
        """Collective: every rank unmaps, then rank 0 removes the segment."""
        import torch.distributed as dist

        dist.barrier()
        self.array = None
        try:
            self.shm.close()
        except BufferError:  # a caller still holds a view; the mapping goes with the process
            pass
        dist.barrier()
        if self.owner:
            self.shm.unlink()
