"""The root's host matrix in shared memory, for one process per GPU on one node.

The reference's drivers keep A on the root and scatter it (MPI_Scatter / Pack + Send; on one
host MPICH moves it through shared memory). The MI355X-node form: rank 0 places A in a POSIX
shared-memory segment, every rank maps it, and each GPU pulls its own shard over its own PCIe
link (Multiplier.distribute_shared). Collective over the default torch.distributed group.
"""
from __future__ import annotations

import os
from multiprocessing import resource_tracker, shared_memory

import numpy as np

from ._lib import check, lib

SHM_DIR = "/dev/shm"


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

    @classmethod
    def create(cls, R: int, C: int, seed: int, tag: str, device: str = "cpu", margin: int = 1 << 30):
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
            if R * C:
                check(lib.mvg_synth_fill_host(me.array.ctypes.data, C, R, C, 0, 0, C, seed), "mvg_synth_fill_host")
        dist.barrier()
        if dist.get_rank() != 0:
            shm = shared_memory.SharedMemory(name=name)
            # only the creator owns (and unlinks) the segment; Python 3.10 registers attachers too
            resource_tracker.unregister(shm._name, "shared_memory")
            me = cls(shm, (R, C), owner=False)
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
