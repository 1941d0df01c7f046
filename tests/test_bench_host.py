"""bench.py's host-side helpers on the CPU (no GPU): the RCCL transport report parser and the
reference-row check every config's y goes through."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN_DIR, REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_parse_rccl_log_transports_and_sizes():
    lines = [
        "host:1234:1240 [0] NCCL INFO comm 0x5555 rank 0 nranks 8 cudaDev 0 busId 1b000 commId 0x1 - Init START",
        "host:1234:1240 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC",
        "host:1234:1240 [0] NCCL INFO Channel 01/0 : 0[1b000] -> 7[e9000] via P2P/IPC read",
        "host:1234:1241 [0] NCCL INFO Channel 00/1 : 0[0] -> 1[0] [send] via NET/Socket/0",
        "host:1234:1240 [0] NCCL INFO comm 0x5555 rank 0 nranks 8 cudaDev 0 busId 1b000 commId 0x1 - Init COMPLETE",
        "host:1234:1240 [0] NCCL INFO comm 0x6666 rank 0 nranks 4 cudaDev 0 busId 1b000 commId 0x2 - Init COMPLETE",
        "unrelated line",
    ]
    r = bench.parse_rccl_log(lines)
    assert r["links"] == {"0->1": ["NET/Socket/0", "P2P/IPC"], "0->7": ["P2P/IPC"]}
    assert r["nranks"] == [8, 4]
    assert len(r["samples"]) == 2 and "via P2P/IPC" in r["samples"][0]
    assert bench.parse_rccl_log([]) == {"links": {}, "nranks": [], "samples": []}


@pytest.mark.parametrize("cfg_name,alg,R,C,n", [("config 3", "colwise", 65536, 65536, 8),
                                                 ("config 4", "blockwise", 131072, 131072, 8),
                                                 ("config 5", "rowwise", 4194304, 512, 1)])
def test_reference_rows_check(cfg_name, alg, R, C, n):
    key = "cfg" + cfg_name.split()[-1]
    with np.load(os.path.join(GOLDEN_DIR, "config_slices.npz")) as z:
        rows, want = z[f"{key}/rows"], z[f"{key}/{alg}/P{n}"]
    y = np.ones(R)
    y[rows] = want
    r = bench.reference_rows_check(cfg_name, alg, R, C, n, y, y.copy())
    assert r["P"] == n and r["rows"] == len(rows) and r["max_rel"] == 0.0 and r["exact_bit_identical"]
    assert ("exact_note" in r) == (alg == "blockwise" and n == 8)  # 2 x 4 grid: arrival-order sums
    # a y off by more than the bar is refused, not reported
    y[rows[0]] *= 1 + 1e-10
    with pytest.raises(AssertionError):
        bench.reference_rows_check(cfg_name, alg, R, C, n, y, None)
    # no reference slice at this P: recorded, not checked — except the row split, whose row sums
    # do not depend on P (its P = 1 slice stands for every P)
    r3 = bench.reference_rows_check(cfg_name, alg, R, C, 3, y, None) if alg != "rowwise" else None
    if r3 is not None:
        assert r3["checked"] is False
    else:
        y[rows[0]] = want[0]
        r = bench.reference_rows_check(cfg_name, alg, R, C, 4, y, None)
        assert r["P"] == 4 and r["max_rel"] == 0.0 and "at P1" in r["source"]


def test_sample_splits_follow_the_reference_checks():
    assert bench._splits("rowwise", 128, 512, 16) and not bench._splits("rowwise", 100, 512, 16)
    assert bench._splits("colwise", 7, 65536, 16) and not bench._splits("colwise", 7, 100, 16)
    assert bench._splits("blockwise", 128, 131072, 16)  # 4 x 4 grid
