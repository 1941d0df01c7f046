"""The executables' one-process-drives-G-GPUs exchange (MVG_NGPUS=G: ncclCommInitAll over G
devices, the grouped ncclCommSplit, every collective issued for all local devices inside one
ncclGroupStart/End per step; csrc/engine.cpp split_steps / exchange_plan / exchange_exact) on a
host without GPUs.

mvg_debug_trace_exchange runs the engine's own exchange code over G stand-in devices with a
recorder in place of RCCL. Each test checks the recorded calls against what the schedule
(mvg_plan_exchange) and the gloo replay (tests/test_distributed_gloo.py) expect: per split
step the members, colours and keys handed to ncclCommSplit; per exchange step one group with
one call per member, all with the same count and root on the same communicator. Then the calls
are executed with numpy on the oracle's local products, in the communicator ranks the splits
define, and rank 0's y must be the reference's: multiplier_rowwise.c:141 (rank-order gather),
multiplier_colwise.c:124 (sum of strips), multiplier_blockwise.c:144-210 (grid-row sums of the
blocks, rows in grid order).
"""
import numpy as np
import pytest

from conftest import max_rel
from matvec_mpi_multiplier_amd import _lib
from matvec_mpi_multiplier_amd import multiplier as mm
from oracle import oracle

SHAPES = {2: (96, 80), 4: (96, 80), 8: (96, 96)}


def _comms(calls):
    """The communicators the split calls create: {split group: {color: [world ranks in comm-rank
    order]}} (members of a colour ordered by key, then world rank, as ncclCommSplit does)."""
    out = {}
    for c in calls:
        if c["kind"] == _lib.XCALL_SPLIT and c["color"] >= 0:
            out.setdefault(c["group"], {}).setdefault(c["color"], []).append((c["key"], c["rank"]))
    return {g: {col: [r for _, r in sorted(m)] for col, m in cols.items()} for g, cols in out.items()}


def _execute(calls, alg, R, C, G, parts):
    """Rank 0's y after running the recorded calls on the local products `parts`."""
    comms = _comms(calls)
    color_of = {(c["group"], c["rank"]): c["color"] for c in calls if c["kind"] == _lib.XCALL_SPLIT}
    bufs = {}
    for r in range(G):
        s = mm.plan_shard(alg, R, C, G, r)
        bufs[r] = {_lib.X_BUF_PART: parts[r].copy(), _lib.X_BUF_ROW: np.zeros(s.y_len), _lib.X_BUF_Y: np.zeros(R),
                   _lib.X_BUF_GATHERED: np.zeros(len(parts[r]) * G)}
    groups = sorted({c["group"] for c in calls if c["kind"] in (_lib.XCALL_GATHER, _lib.XCALL_REDUCE)})
    for g in groups:
        step = [c for c in calls if c["group"] == g]
        assert {c["kind"] for c in step} in ({_lib.XCALL_GATHER}, {_lib.XCALL_REDUCE}), step
        # per communicator of this step: its members' calls
        by_comm = {}
        for c in step:
            if c["comm"] == -1:
                members = list(range(G))
            else:
                members = comms[c["comm"]][color_of[(c["comm"], c["rank"])]]
            by_comm.setdefault(tuple(members), []).append(c)
        for members, cs in by_comm.items():
            assert sorted(c["rank"] for c in cs) == sorted(members), (members, cs)  # every member, once
            assert len({c["count"] for c in cs}) == 1 and len({c["root"] for c in cs}) == 1, cs
            root = members[cs[0]["root"]]
            n = cs[0]["count"]
            srcs = {c["rank"]: bufs[c["rank"]][c["src"]][:n] for c in cs}
            dst = next(c["dst"] for c in cs if c["rank"] == root)
            if cs[0]["kind"] == _lib.XCALL_GATHER:
                bufs[root][dst][: n * len(members)] = np.concatenate([srcs[m] for m in members])
            else:
                bufs[root][dst][:n] = np.sum([srcs[m] for m in members], axis=0)
    for c in calls:
        if c["kind"] == _lib.XCALL_COMBINE:
            assert c["rank"] == 0 and c["group"] == -1
            gathered = bufs[0][c["src"]].reshape(G, -1)
            if alg == "colwise":
                bufs[0][c["dst"]][:] = gathered.sum(axis=0)
            else:  # grid row i: its blocks' partials
                gr, gc = mm.get_2_most_closest_multipliers(G)
                bufs[0][c["dst"]][:] = np.concatenate([gathered[i * gc:(i + 1) * gc].sum(axis=0) for i in range(gr)])
    return bufs[0][_lib.X_BUF_Y]


def _parts(alg, R, C, G, A, x):
    out = []
    for r in range(G):
        s = mm.plan_shard(alg, R, C, G, r)
        blk = A[s.row_off:s.row_off + s.n_rows, s.col_off:s.col_off + s.n_cols]
        out.append(oracle.multiply_std_rowwise(blk, x[s.col_off:s.col_off + s.n_cols]))
    return out


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
@pytest.mark.parametrize("exact", [False, True])
def test_single_process_exchange_computes_the_reference_y(G, alg, exact):
    R, C = SHAPES[G]
    A, x = oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0]
    calls = mm.trace_exchange(alg, R, C, G, exact=exact)
    y = _execute(calls, alg, R, C, G, _parts(alg, R, C, G, A, x))
    want = oracle.multiply_std_rowwise(A, x)
    assert max_rel(y, want) <= 1e-13, max_rel(y, want)
    if alg == "rowwise":
        np.testing.assert_array_equal(y, want)  # a gather moves the row sums unchanged


@pytest.mark.parametrize("G", [2, 4, 8])
def test_single_process_block_split_communicators(G):
    """The block split's grouped ncclCommSplit (engine.cpp split_steps) and collectives on the
    utils.c:26-37 grid: per grid row a communicator of its c ranks (colour = grid row, key = grid
    column) reducing R/r doubles to the row leader, then the grid-column-0 leaders (colour 0,
    key = grid row; everyone else NCCL_SPLIT_NOCOLOR) gathering to rank 0 — every split and
    every collective of a step issued in one group by all G local devices."""
    R, C = SHAPES[G]
    gr, gc = mm.get_2_most_closest_multipliers(G)
    calls = mm.trace_exchange("blockwise", R, C, G)
    plans = [mm.plan_exchange("blockwise", R, C, G, r) for r in range(G)]
    splits = [c for c in calls if c["kind"] == _lib.XCALL_SPLIT]
    split_groups = sorted({c["group"] for c in splits})
    # one group per split step, every device calling ncclCommSplit in it (on the world comm)
    nsplit = sum(1 for st in plans[0] if st.comm != _lib.X_WORLD)
    assert len(split_groups) == nsplit
    for g in split_groups:
        cs = [c for c in splits if c["group"] == g]
        assert sorted(c["rank"] for c in cs) == list(range(G)) and all(c["comm"] == -1 for c in cs)
    comms = _comms(calls)
    if gr > 1 and gc > 1:
        row_g, lead_g = split_groups
        assert comms[row_g] == {i: [i * gc + j for j in range(gc)] for i in range(gr)}
        assert comms[lead_g] == {0: [i * gc for i in range(gr)]}
        for c in splits:
            if c["group"] == lead_g and c["rank"] % gc != 0:
                assert c["color"] == -1  # not a leader: NCCL_SPLIT_NOCOLOR
    # the collectives: counts and roots as the schedule says, each step in one group
    xs = [c for c in calls if c["kind"] != _lib.XCALL_SPLIT]
    steps = sorted({c["group"] for c in xs})
    assert len(steps) == len(plans[0])
    for k, g in enumerate(steps):
        for c in (c for c in xs if c["group"] == g):
            st = plans[c["rank"]][k]
            assert st.member and c["count"] == st.count == R // gr and c["root"] == st.root == 0
            assert c["kind"] == (_lib.XCALL_REDUCE if st.op == _lib.X_REDUCE else _lib.XCALL_GATHER)
        members = {c["rank"] for c in xs if c["group"] == g}
        assert members == {r for r in range(G) if plans[r][k].member}


def test_single_process_exact_exchange_gathers_in_rank_order():
    """Exact mode: one world ncclGather of every partial into rank 0's gather buffer (rank order),
    then the combine kernel on rank 0, outside the group."""
    calls = mm.trace_exchange("colwise", 64, 64, 4, exact=True)
    g = [c for c in calls if c["kind"] == _lib.XCALL_GATHER]
    assert sorted(c["rank"] for c in g) == [0, 1, 2, 3] and {c["count"] for c in g} == {64}
    assert next(c for c in g if c["rank"] == 0)["dst"] == _lib.X_BUF_GATHERED
    (comb,) = [c for c in calls if c["kind"] == _lib.XCALL_COMBINE]
    assert comb["rank"] == 0 and comb["count"] == 4 * 64 and comb["dst"] == _lib.X_BUF_Y
    assert mm.trace_exchange("rowwise", 64, 64, 1) == []  # one device: no exchange at all
