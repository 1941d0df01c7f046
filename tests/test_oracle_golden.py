"""The oracle (oracle/cpu_ref.c) against the golden vectors the REAL reference produced.

This pins the oracle before anything is checked against it: wherever the reference is
deterministic the restatement must be bit-exact; block split with >= 3 grid columns takes
its partials in MPI_ANY_SOURCE arrival order (multiplier_blockwise.c:187,206), so there the
bar is 1e-15 relative per element.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR, case_inputs, golden_runs, max_rel
from oracle import oracle, ref_runner


def _runs():
    import json

    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        man = json.load(f)
    return [(c, a, p) for c, a, p in golden_runs(man)]


@pytest.mark.parametrize("case,alg,p", _runs(), ids=lambda v: v["name"] if isinstance(v, dict) else str(v))
def test_oracle_matches_reference(golden, case, alg, p):
    A, x = case_inputs(case)
    y_ref = golden[f"{case['name']}/{alg}/P{p}"]
    y = oracle.multiply(alg, A, x, p)
    gr, gc = oracle.grid_shape(p)
    if alg == "blockwise" and gc >= 3:
        assert max_rel(y, y_ref) <= 1e-15
    else:
        np.testing.assert_array_equal(y, y_ref)


def test_fixture_expected_values(golden):
    # the 4x8 fixture's y, as every reference executable prints it
    expect = np.array([222.19999999999999, 196.55000000000001, 191.56999999999999, 232.90000000000001])
    for key, y in golden.items():
        if key.startswith("fixture_4x8/"):
            np.testing.assert_array_equal(y, expect)


def test_golden_covers_every_algorithm_and_rank_count(manifest):
    seen = {(a, p) for _, a, p in golden_runs(manifest)}
    for alg in ("rowwise", "colwise", "blockwise"):
        assert {1, 2, 4, 8} <= {p for a, p in seen if a == alg}


def test_synthetic_values_roundtrip_through_reference_text_format():
    # every synthetic value is k/10000; "%.4f" text of it parses back (strtod == fscanf %lf)
    # to the same double, so synthetic and text inputs are interchangeable bit for bit.
    k = np.arange(10000)
    v = k / 10000.0
    back = np.array([float(f"{t:.4f}") for t in v])
    np.testing.assert_array_equal(v, back)
    vals = np.array([oracle.synth_value(42, i) for i in range(20000)])
    np.testing.assert_array_equal(vals, np.round(vals * 10000) / 10000.0)
    assert vals.min() >= 0.0 and vals.max() <= 0.9999


def test_oracle_grid_shape_is_reference_factorisation():
    # utils.c:26-37: rows = largest divisor <= sqrt(p)
    expect = {1: (1, 1), 2: (1, 2), 4: (2, 2), 6: (2, 3), 8: (2, 4), 12: (3, 4), 24: (4, 6), 7: (1, 7), 9: (3, 3)}
    for p, rc in expect.items():
        assert oracle.grid_shape(p) == rc


def test_oracle_rowwise_independent_of_p():
    A, x = oracle.synth(48, 33, 42), oracle.synth(1, 33, 4242)[0]
    y1 = oracle.multiply("rowwise", A, x, 1)
    for p in (2, 3, 4, 6, 8, 12, 16, 24, 48):
        np.testing.assert_array_equal(oracle.multiply("rowwise", A, x, p), y1)


def test_oracle_refuses_indivisible():
    A, x = oracle.synth(6, 10, 42), oracle.synth(1, 10, 4242)[0]
    with pytest.raises(ValueError):
        oracle.multiply("rowwise", A, x, 4)
    with pytest.raises(ValueError):
        oracle.multiply("colwise", A, x, 3)
    with pytest.raises(ValueError):
        oracle.multiply("blockwise", A, x, 3)  # 1x3 grid: 60 % 3 == 0 but 10 % 3 != 0


def test_oracle_timing_harness_returns_reference_y():
    A, x = oracle.synth(64, 96, 42), oracle.synth(1, 96, 4242)[0]
    for alg in ("rowwise", "colwise", "blockwise"):
        t, y = oracle.time_multiply(alg, A, x, 4, 3)
        assert t > 0
        np.testing.assert_array_equal(y, oracle.multiply(alg, A, x, 4))


@pytest.mark.skipif(not all(ref_runner.available(a) for a in ("rowwise", "colwise", "blockwise")),
                    reason="oracle/_ref (the reference built from its sources) or mpiexec absent")
def test_ref_runner_real_reference_matches_oracle():
    # bench.py's cpu_baseline leg runs the real reference through this runner on the GPU box;
    # its y must be the oracle's (bit for bit for row split; col/block: MPI reduction order)
    R, C, P = 32, 256, 4
    A, x = oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0]
    for alg in ("rowwise", "colwise", "blockwise"):
        r = ref_runner.run(alg, R, C, P, timeout=120)
        assert r["seconds"] > 0
        want = oracle.multiply(alg, A, x, P)
        if alg == "rowwise":
            np.testing.assert_array_equal(r["y"], want)
        else:
            np.testing.assert_allclose(r["y"], want, rtol=1e-15)


# ---- BASELINE configs 2-5 at their own (R, C, P): the reference's y on bands of each config's
# rows (tests/golden/make_config_slices.py). The oracle on the same rows at the same P must give
# the reference's bits (block split over > 2 grid columns: its arrival order, 1e-15).
def _slice_runs():
    with open(os.path.join(GOLDEN_DIR, "config_slices.json")) as f:
        meta = json.load(f)
    return [(c["name"], c["alg"], c["R"], c["C"], int(p[1:])) for c in meta["configs"] for p in c["runs"]]


import json  # noqa: E402


@pytest.mark.parametrize("cfg,alg,R,C,p", _slice_runs())
def test_oracle_matches_reference_on_config_rows(cfg, alg, R, C, p):
    with np.load(os.path.join(GOLDEN_DIR, "config_slices.npz")) as z:
        rows, want = z[f"{cfg}/rows"], z[f"{cfg}/{alg}/P{p}"]
    bands = np.split(rows, np.flatnonzero(np.diff(rows) != 1) + 1)
    A = np.vstack([oracle.synth_block(int(b[0]), len(b), 0, C, C, 42) for b in bands])
    x = oracle.synth(1, C, 4242)[0]
    y = oracle.multiply(alg, A, x, p)
    if alg == "blockwise" and oracle.grid_shape(p)[1] >= 3:
        assert max_rel(y, want) <= 1e-15
    else:
        np.testing.assert_array_equal(y, want)


def test_config_slices_cover_every_baseline_config_and_gpu_count():
    runs = {(cfg, p) for cfg, _, _, _, p in _slice_runs()}
    assert {("cfg2", 1), ("cfg2", 8), ("cfg5", 8)} <= runs
    for cfg in ("cfg3", "cfg4"):
        assert {(cfg, p) for p in (1, 2, 4, 8)} <= runs
