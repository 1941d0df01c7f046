"""Worker for tests/test_gpu_rank_mode.py (run under torch.distributed.run; not collected by pytest).

One process per rank, every rank on GPU 0 (on a one-GPU box RCCL needs a distinct NCCL_HOSTID
per rank and loopback sockets, as bench.py's MVG_SAME_DEVICE rehearsal does). For each
algorithm: distribute(A1, x1) -> multiply -> distribute(A2, x2) -> multiply -> collect, with
no engine sync in between. The root's second distribute overwrites dA/dx (own shard) and the
staging buffers (peer sends) while the first multiply's GEMV and exchange may still be in
flight, so y equals A2·x2 only if the engine orders those copies after them.
Prints one JSON line per algorithm on rank 0.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

rank = int(os.environ.get("RANK", "0"))
world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    os.environ.setdefault("NCCL_HOSTID", f"mvg-b2b-{rank}")
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    R, C = int(sys.argv[1]), int(sys.argv[2])
    dist.init_process_group("gloo")
    comm = mm.Comm.from_process_group(0)
    A1, x1 = oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0]
    A2, x2 = oracle.synth(R, C, 7), oracle.synth(1, C, 77)[0]
    ok = True
    try:
        for alg in ("rowwise", "colwise", "blockwise"):
            with mm.Multiplier(alg, R, C, comm) as e:
                root = e.is_root()
                e.distribute(A1 if root else None, x1 if root else None)
                e.multiply()
                e.distribute(A2 if root else None, x2 if root else None)
                e.multiply()
                y = e.collect()
            if root:
                want = oracle.multiply(alg, A2, x2, world)
                rel = float(np.max(np.abs(y - want) / np.abs(want)))
                ok &= rel <= 1e-12
                print(json.dumps({"alg": alg, "world": world, "R": R, "C": C, "max_rel": rel}), flush=True)
    finally:
        comm.destroy()
        dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
