"""One-process-per-GPU engine paths run back to back without an engine sync:
distribute -> multiply -> distribute -> multiply -> collect must give A2·x2, at world size 1
(every device pulls its own shard) and at world size 2 with both ranks on GPU 0 (the root
stages its peer's shard and ncclSends it; its own shard is copied on the copy stream, which
must wait for the previous GEMV still reading dA/dx)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "rank_worker_b2b.py")


def run_worker(nproc: int, R: int, C: int):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), WORKER, str(R), str(C)],
                       env=dict(os.environ), capture_output=True, text=True, timeout=110)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


@pytest.mark.parametrize("nproc,R,C", [(1, 640, 2048), (2, 640, 2048), (2, 96, 131072)])
def test_back_to_back_distribute_without_sync(nproc, R, C):
    r, lines = run_worker(nproc, R, C)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert sorted(l["alg"] for l in lines) == ["blockwise", "colwise", "rowwise"]
    for l in lines:
        assert l["world"] == nproc and l["max_rel"] <= 1e-12, l
