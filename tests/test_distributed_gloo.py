"""The N > 1 path on CPU: world_size 2, 4 and 8 over torch.distributed `gloo`.

Each rank takes its shard from the C planner (mvg_plan_shard), computes its local product
(with the oracle standing in for the GPU kernel — there is no GPU here), then runs the exchange
step exactly as the C engine does: the same schedule from mvg_plan_exchange (gather / reduce,
world / grid-row / leader communicators, buffers, roots), executed with gloo collectives instead
of RCCL. Rank 0's y must equal the reference's golden y at that P. Also covers the 128-byte
RCCL unique-id bootstrap that bench.py runs over the default process group.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN_DIR, REPO, max_rel

CASES = [
    # (case, R, C, alg, P, exact)
    ("fixture_4x8", 4, 8, "rowwise", 2, True),
    ("fixture_4x8", 4, 8, "colwise", 2, True),
    ("fixture_4x8", 4, 8, "blockwise", 2, True),
    ("fixture_4x8", 4, 8, "rowwise", 4, True),
    ("fixture_4x8", 4, 8, "colwise", 4, False),
    ("fixture_4x8", 4, 8, "blockwise", 4, True),
    ("sq_480", 480, 480, "rowwise", 2, True),
    ("sq_480", 480, 480, "colwise", 2, True),
    ("sq_480", 480, 480, "blockwise", 2, True),
    ("sq_480", 480, 480, "colwise", 4, False),
    ("sq_480", 480, 480, "blockwise", 4, True),
    ("wide_120x6000", 120, 6000, "blockwise", 4, True),
    ("tall_960x96", 960, 96, "rowwise", 4, True),
    # world size 8: the column split's 8 strips and the block split's 2 x 4 grid (config 4's
    # grid, utils.c:26-37): grid-row Reduce over 4 ranks, then the leaders' Gather
    # (multiplier_blockwise.c:144-210)
    ("fixture_4x8", 4, 8, "colwise", 8, False),
    ("fixture_4x8", 4, 8, "blockwise", 8, False),
    ("sq_480", 480, 480, "rowwise", 8, True),
    ("sq_480", 480, 480, "colwise", 8, False),
    ("sq_480", 480, 480, "blockwise", 8, False),
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(case, R, C):
    from oracle import oracle

    if case.startswith("fixture"):
        A = np.loadtxt(os.path.join(GOLDEN_DIR, "matrix_4_8.txt")).reshape(4, 8)
        x = np.loadtxt(os.path.join(GOLDEN_DIR, "vector_8.txt"))
        return A, x
    return oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0]


def _worker(rank, world, port, case, R, C, alg, outq):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd import _lib
    from matvec_mpi_multiplier_amd import multiplier as mm
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # --- bootstrap: rank 0's 128-byte id reaches every rank unchanged
        fake = bytes((i * 7 + 3) % 256 for i in range(_lib.UNIQUE_ID_BYTES))
        uid = mm.broadcast_unique_id(lambda: fake)
        assert uid == fake

        # --- local product on this rank's shard
        A, x = _inputs(case, R, C)
        s = mm.plan_shard(alg, R, C, world, rank)
        blk = A[s.row_off:s.row_off + s.n_rows, s.col_off:s.col_off + s.n_cols]
        part = oracle.multiply_std_rowwise(blk, x[s.col_off:s.col_off + s.n_cols])
        bufs = {_lib.X_BUF_PART: torch.from_numpy(part.copy()),
                _lib.X_BUF_ROW: torch.zeros(s.y_len, dtype=torch.float64),
                _lib.X_BUF_Y: torch.zeros(R, dtype=torch.float64)}

        # --- the exchange schedule, as the C engine runs it over RCCL
        plans = [mm.plan_exchange(alg, R, C, world, r) for r in range(world)]
        nsteps = len(plans[rank])
        assert all(len(p) == nsteps for p in plans)
        for k in range(nsteps):
            st = plans[rank][k]
            # communicator = members of this step with the same color, ordered by key
            groups = {}
            for r in range(world):
                o = plans[r][k]
                if o.member:
                    groups.setdefault(o.color, []).append((o.key, r))
            handles = {}
            for color in sorted(groups):  # every rank creates every group, same order
                ranks = [r for _, r in sorted(groups[color])]
                handles[color] = (ranks, dist.new_group(ranks) if st.comm != _lib.X_WORLD else None)
            if not st.member:
                continue
            ranks, g = handles[st.color]
            root = ranks[st.root]
            src = bufs[st.src]
            assert src.numel() == st.count
            if st.op == _lib.X_GATHER:
                gl = [torch.empty(st.count, dtype=torch.float64) for _ in ranks] if rank == root else None
                dist.gather(src, gather_list=gl, dst=root, group=g)
                if rank == root:
                    bufs[st.dst][: st.count * len(ranks)] = torch.cat(gl)
            else:
                t = src.clone()
                dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, group=g)
                if rank == root:
                    bufs[st.dst][: st.count] = t
        if rank == 0:
            outq.put(bufs[_lib.X_BUF_Y].numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,R,C,alg,P,exact", CASES)
def test_gloo_exchange_replay_matches_reference(golden, case, R, C, alg, P, exact):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, P, port, case, R, C, alg, q)) for r in range(P)]
    for p in procs:
        p.start()
    y = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = golden[f"{case}/{alg}/P{P}"]
    if exact:
        np.testing.assert_array_equal(y, want)
    else:  # gloo's reduce order for > 2 ranks is its own (MPICH/RCCL differ too)
        assert max_rel(y, want) <= 1e-15


def _shm_worker(rank, world, port, R, C, outq):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd.hostshare import SharedHostMatrix
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from matvec_mpi_multiplier_amd.hostshare import fill_threads

        had = os.environ.get("MVG_THREADS")
        sh = SharedHostMatrix.create(R, C, 42, f"test_{port}", margin=0, threads=fill_threads(world))
        assert sh is not None
        assert os.environ.get("MVG_THREADS") == had  # the rank's fill threads were set for the fill only
        # every rank sees rank 0's synthetic matrix; each checks the rows its shard would pull
        lo, hi = rank * R // world, (rank + 1) * R // world
        np.testing.assert_array_equal(sh.array[lo:hi], oracle.synth_block(lo, hi - lo, 0, C, C, 42))
        # the bench's host_memory record: every rank's share gathered on every rank (all_gather_object)
        rec = bench.host_setup_record({**sh.timing, "pin_bytes": 8 * (hi - lo) * C, "pin_s": 0.001}, True, C)
        assert [r["rows"] for r in rec["by_rank"]] == [R * (q + 1) // world - R * q // world for q in range(world)]
        assert sum(r["rows"] for r in rec["by_rank"]) == R and rec["rows"] == R
        assert all(r["threads"] == fill_threads(world) and r["fill_s"] >= 0 for r in rec["by_rank"])
        assert rec["pin_bytes"] == 8 * R * C and rec["pin_GBps"] is not None  # (a 96 x 80 fill rounds to 0 s)
        sh.close()
        outq.put((rank, "ok"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stale", [False, True])
def test_shared_host_matrix_two_ranks(stale):
    """bench.py's end-to-end `shared` distribution: rank 0 creates the root's A in /dev/shm,
    rank 1 maps the same bytes, each fills its share with its share of the CPUs, both unmap, the
    segment is removed (no leak), and the bench's per-rank setup record adds up. A segment of the
    same name left by a killed run is replaced, not fatal."""
    from multiprocessing import resource_tracker, shared_memory

    from matvec_mpi_multiplier_amd.hostshare import shm_free_bytes

    if shm_free_bytes() < (64 << 20):
        pytest.skip("/dev/shm too small here")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    if stale:
        old = shared_memory.SharedMemory(name=f"mvg_test_{port}", create=True, size=4096)
        resource_tracker.unregister(old._name, "shared_memory")  # left behind on purpose
        old.close()
    procs = [ctx.Process(target=_shm_worker, args=(r, 2, port, 96, 80, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [(0, "ok"), (1, "ok")]
    assert not os.path.exists(f"/dev/shm/mvg_test_{port}")


def _exact_worker(rank, world, port, case, R, C, alg, outq):
    """The exact-mode exchange (engine.cpp exchange_exact) over gloo: every rank's partial
    gathered to rank 0 in rank order, then added there in the reference's order — MPICH's
    MPI_Reduce tree for the column split (binomial, or reduce-scatter + gather for buffers over
    2 KiB), the grid row's partials into a zeroed y in rank order for the block split (the order
    of the combine kernels in csrc/gemv_exact.hip)."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd import multiplier as mm
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        A, x = _inputs(case, R, C)
        s = mm.plan_shard(alg, R, C, world, rank)
        blk = A[s.row_off:s.row_off + s.n_rows, s.col_off:s.col_off + s.n_cols]
        part = torch.from_numpy(oracle.multiply_std_rowwise(blk, x[s.col_off:s.col_off + s.n_cols]).copy())
        gl = [torch.empty_like(part) for _ in range(world)] if rank == 0 else None
        dist.gather(part, gather_list=gl, dst=0)
        if rank == 0:
            parts = [g.numpy().copy() for g in gl]
            if alg == "colwise":
                y = oracle.mpich_reduce(parts)
            else:
                gr, gc = mm.get_2_most_closest_multipliers(world)
                lr = R // gr
                y = np.zeros(R)
                for r in range(world):
                    y[(r // gc) * lr:(r // gc + 1) * lr] = y[(r // gc) * lr:(r // gc + 1) * lr] + parts[r]
            outq.put(y)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,R,C,alg,P", [
    ("fixture_4x8", 4, 8, "colwise", 4), ("sq_480", 480, 480, "colwise", 4), ("sq_480", 480, 480, "colwise", 3),
    ("sq_480", 480, 480, "blockwise", 4), ("wide_120x6000", 120, 6000, "blockwise", 2),
    # world size 8 (config 3's largest P, config 4's 2 x 4 grid)
    ("fixture_4x8", 4, 8, "colwise", 8), ("sq_480", 480, 480, "colwise", 8), ("fixture_4x8", 4, 8, "blockwise", 8),
    ("sq_480", 480, 480, "blockwise", 8),
    # MPICH's reduce-scatter + gather order (R * 8 > 2048 bytes) where it differs from the
    # binomial tree, and the binomial tree at a non-power-of-two P for a short y
    ("sq_720", 720, 720, "colwise", 5), ("sq_720", 720, 720, "colwise", 10), ("wide_120x6000", 120, 6000, "colwise", 5),
])
def test_gloo_exact_exchange_is_bit_identical_to_reference(golden, case, R, C, alg, P):
    # where the RCCL/gloo reduce differs from MPICH in the last bit (the replay above at P = 4),
    # the exact exchange gives the reference's own bits; a block split over more than two grid
    # columns adds in the reference's message-arrival order (blockwise.c:187,206): there the
    # exchange gives the oracle's rank order bit for bit and the reference's y within 1e-15
    from oracle import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exact_worker, args=(r, P, port, case, R, C, alg, q)) for r in range(P)]
    for p in procs:
        p.start()
    y = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = golden[f"{case}/{alg}/P{P}"]
    if alg == "blockwise" and oracle.grid_shape(P)[1] > 2:
        A, x = _inputs(case, R, C)
        np.testing.assert_array_equal(y, oracle.multiply(alg, A, x, P))
        assert max_rel(y, want) <= 1e-15
    else:
        np.testing.assert_array_equal(y, want)
