"""Parity of the HIP path (called through the C-ABI) with the reference.

Bar (BASELINE.json north_star): <= 1e-12 relative per element against the reference on the
same inputs — the GPU sums in a different (fixed) order than the reference's sequential
loop. Checked against (a) the golden vectors the real reference produced, (b) the pinned
oracle on the same seeded inputs, and (c) at the full BASELINE sizes: every row of y at
configs 2, 3, 4 and 5 whole (config 4: 128 GiB on one GPU) and at their per-GPU shards against
the oracle (tree within the bar, exact bit for bit), plus size-independent properties (exact
scaling by 2, run-to-run bit determinism).
"""
import os

import numpy as np
import pytest

from conftest import REPO as REPO_ROOT, case_inputs, golden_runs, max_rel
from matvec_mpi_multiplier_amd import _lib
from matvec_mpi_multiplier_amd import multiplier as mm
from oracle import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-12


@pytest.fixture(scope="module")
def comm1():
    assert mm.device_count() >= 1, "no GPU visible"
    c = mm.Comm.init_all([0])
    yield c
    c.destroy()


def exact_dot(A, x):
    """Correctly rounded-ish reference: fp64 products summed with math.fsum (exact sum)."""
    import math

    return np.array([math.fsum(A[i] * x) for i in range(A.shape[0])])


# ---------------------------------------------------------------- the raw kernel
SHAPES = [(1, 1), (1, 2), (3, 5), (4, 8), (5, 7), (63, 129), (64, 128), (65, 127), (257, 1000), (1000, 257),
          (33, 4096), (7, 20001), (2049, 512), (100, 1), (100, 2), (100, 3),
          (5, 40000), (130, 16388), (3, 65538)]


@pytest.mark.parametrize("m,k", SHAPES)
def test_gemv_all_variants_vs_oracle(m, k):
    A = oracle.synth(m, k, 42)
    x = oracle.synth(1, k, 4242)[0]
    y_ref = oracle.multiply_std_rowwise(A, x)
    for v in range(_lib.lib.mvg_gemv_variant_count()):
        name = _lib.lib.mvg_gemv_variant_name(v).decode()
        # an odd k is an odd lda here: the 16-B kernels read every other row 8 bytes off a
        # 16-B boundary (unaligned vector loads) and must give the same result
        y = mm.multiply_std_rowwise(A, x, variant=v)
        assert max_rel(y, y_ref) <= TOL, (name, m, k)


@pytest.mark.parametrize("m,k", [(5, 7), (65, 127), (257, 1000), (33, 4096), (130, 16388), (2049, 512), (3, 65538)])
def test_gemv_all_variants_on_signed_data(m, k):
    """Mixed-sign inputs (cancellation): the relative bar per element is ill-conditioned there, so
    the tree-summed kernels are held to the forward-error bound of a sum of k products,
    |y - y_ref| <= 1e-13 * sum_j |a_ij x_j| per row (k * eps * sum|.| is 1.5e-12 at k = 65538; the
    fixed-order tree does far better), against the reference's sequential sums (the oracle)."""
    rng = np.random.default_rng(m * 7919 + k)
    A = rng.uniform(-1.0, 1.0, size=(m, k))
    x = rng.uniform(-1.0, 1.0, size=k)
    y_ref = oracle.multiply_std_rowwise(A, x)
    scale = np.abs(A) @ np.abs(x)
    for v in range(_lib.lib.mvg_gemv_variant_count()):
        name = _lib.lib.mvg_gemv_variant_name(v).decode()
        y = mm.multiply_std_rowwise(A, x, variant=v)
        err = float(np.max(np.abs(y - y_ref) / scale))
        assert err <= 1e-13, (name, m, k, err)
    # the exact kernels: the reference's own bits, signs or not
    assert np.array_equal(mm.multiply_std_rowwise(A, x, exact=True), y_ref), (m, k)


def test_gemv_16b_kernels_on_views_off_16b():
    # A and x starting 8 bytes into their buffers (an offset view), odd and even lda
    for m, k, lda in [(70, 300, 301), (130, 4096, 4097), (9, 20001, 20002), (257, 1000, 1000)]:
        full = oracle.synth(m, lda + 1, 42)
        x = oracle.synth(1, k + 1, 4242)[0]
        dA, dx, dy = mm.DeviceBuffer(m * (lda + 1)).upload(full), mm.DeviceBuffer(k + 1).upload(x), mm.DeviceBuffer(m)
        view = full.reshape(-1)[1 + np.arange(m)[:, None] * lda + np.arange(k)[None, :]]  # rows at 8 + lda*8*r
        want = oracle.multiply_std_rowwise(view, x[1:k + 1])
        for v in range(_lib.lib.mvg_gemv_variant_count()):
            mm.gemv(dA.ptr + 8, lda, dx.ptr + 8, dy.ptr, m, k, None, v)
            _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
            assert max_rel(dy.download(), want) <= TOL, (_lib.lib.mvg_gemv_variant_name(v).decode(), m, k, lda)


def test_gemv_padded_lda_and_offsets():
    # a sub-block view (lda > k), as a block shard inside a bigger row-major matrix would be
    m, k, lda = 70, 300, 512
    full = oracle.synth(m, lda, 42)
    x = oracle.synth(1, k, 4242)[0]
    dA, dx, dy = mm.DeviceBuffer(m * lda).upload(full), mm.DeviceBuffer(k).upload(x), mm.DeviceBuffer(m)
    for v in range(_lib.lib.mvg_gemv_variant_count()):
        mm.gemv(dA.ptr, lda, dx.ptr, dy.ptr, m, k, None, v)
        _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
        assert max_rel(dy.download(), oracle.multiply_std_rowwise(full[:, :k], x)) <= TOL


def test_gemv_k_zero_writes_zeros_and_m_zero_is_noop():
    dy = mm.DeviceBuffer(16).upload(np.full(16, 7.0))
    dA, dx = mm.DeviceBuffer(16), mm.DeviceBuffer(16)
    mm.gemv(dA.ptr, 0, dx.ptr, dy.ptr, 16, 0)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    np.testing.assert_array_equal(dy.download(), np.zeros(16))  # the reference's `sum = 0`
    dy.upload(np.full(16, 7.0))
    mm.gemv(dA.ptr, 1, dx.ptr, dy.ptr, 0, 1)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    np.testing.assert_array_equal(dy.download(), np.full(16, 7.0))


def test_gemv_rejects_bad_arguments():
    d = mm.DeviceBuffer(8)
    for args in [(d.ptr, 1, d.ptr, d.ptr, 2, 4), (d.ptr, 4, d.ptr, d.ptr, -1, 4), (None, 4, d.ptr, d.ptr, 2, 4)]:
        with pytest.raises(_lib.MvgError):
            mm.gemv(*args)


@pytest.mark.parametrize("lda_mult", [1, 2])
def test_one_row_form_runs_in_1_gib_launches_with_ragged_tail(lda_mult):
    # short rows (one row per wave) reading more than 1 GiB go out as launches of <= 1 GiB of
    # the bytes read (gemv.hip kOneRowLaunchBytes; a view's wider lda does not shrink them): rows
    # on both sides of each piece boundary and the ragged last piece must match the oracle, and
    # the auto path must equal the explicit variant
    k = 300
    lda = k * lda_mult
    piece = (1 << 30) // (8 * k) // 4 * 4  # rows per launch: 1 GiB read, whole 4-row workgroups
    m = 2 * piece + 37
    v = _lib.lib.mvg_gemv_auto_variant(lda, m, k)
    assert _lib.lib.mvg_gemv_variant_name(v).decode() == "vec_l64_r1_u4_nt1_o5"
    dA, dx, dy = mm.DeviceBuffer(m * lda), mm.DeviceBuffer(k), mm.DeviceBuffer(m)
    _lib.check(_lib.lib.mvg_synth_fill_device(dA.ptr, lda, m, lda, 0, 0, lda, 42, None), "fill A")
    x = oracle.synth(1, k, 4242)[0]
    dx.upload(x)
    mm.gemv(dA.ptr, lda, dx.ptr, dy.ptr, m, k)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    y = dy.download()
    rows = (0, piece - 3, 2 * piece - 3, m - 40)
    wants = [oracle.multiply_std_rowwise(oracle.synth_block(r0, 40, 0, k, lda, 42), x) for r0 in rows]
    for r0, want in zip(rows, wants):
        assert max_rel(y[r0:r0 + 40], want) <= TOL, r0
    assert y.min() >= 0 and y.max() <= k * 0.9999 * 0.9999
    mm.gemv(dA.ptr, lda, dx.ptr, dy.ptr, m, k, None, v)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    np.testing.assert_array_equal(dy.download(), y)
    # the exact kernels split short rows the same way (gemv_exact.hip kShortRowLaunchBytes)
    _lib.check(_lib.lib.mvg_gemv_exact(dA.ptr, lda, dx.ptr, dy.ptr, m, k, None), "exact")
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    ye = dy.download()
    for r0, want in zip(rows, wants):
        np.testing.assert_array_equal(ye[r0:r0 + 40], want, err_msg=str(r0))


def test_gemv_error_vs_exact_sum_not_worse_than_reference():
    # the GPU's fixed-order FMA tree is at least as accurate as the sequential sum
    A = oracle.synth(64, 65536, 42)
    x = oracle.synth(1, 65536, 4242)[0]
    y_gpu = mm.multiply_std_rowwise(A, x)
    y_seq = oracle.multiply_std_rowwise(A, x)
    y_ex = exact_dot(A, x)
    assert max_rel(y_gpu, y_ex) <= max(max_rel(y_seq, y_ex), 1e-15)
    assert max_rel(y_gpu, y_seq) <= TOL


def test_device_synth_fill_bit_exact():
    R, Cn = 333, 1027
    d = mm.DeviceBuffer(R * Cn)
    _lib.check(_lib.lib.mvg_synth_fill_device(d.ptr, Cn, R, Cn, 0, 0, Cn, 42, None), "fill")
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    np.testing.assert_array_equal(d.download().reshape(R, Cn), oracle.synth(R, Cn, 42))
    # a shard of a huge global matrix (64-bit global index)
    GC = 131072
    _lib.check(_lib.lib.mvg_synth_fill_device(d.ptr, 100, 50, 100, 70000, 130900, GC, 42, None), "fill")
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    got = d.download(50 * 100).reshape(50, 100)
    np.testing.assert_array_equal(got, oracle.synth_block(70000, 50, 130900, 100, GC, 42))


# ---------------------------------------------------------------- engine vs golden (P = 1)
def _golden_p1(manifest):
    return [(c, a, p) for c, a, p in golden_runs(manifest) if p == 1]


def test_engine_p1_matches_reference_golden(comm1, golden, manifest):
    for case, alg, p in _golden_p1(manifest):
        A, x = case_inputs(case)
        with mm.Multiplier(alg, case["R"], case["C"], comm1) as e:
            e.distribute(A, x)
            e.multiply()
            y = e.collect()
        key = f"{case['name']}/{alg}/P1"
        assert max_rel(y, golden[key]) <= TOL, key
        assert max_rel(y, oracle.multiply(alg, A, x, 1)) <= TOL


@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
def test_engine_forced_collectives_p1(alg, monkeypatch, golden):
    # MVG_ALWAYS_COLLECT=1 runs the RCCL exchange (ncclGather / ncclReduce / ncclCommSplit)
    # even with one rank, so the collective code path executes on a one-GPU box.
    monkeypatch.setenv("MVG_ALWAYS_COLLECT", "1")
    c = mm.Comm.init_all([0])
    try:
        A, x = oracle.synth(480, 480, 42), oracle.synth(1, 480, 4242)[0]
        with mm.Multiplier(alg, 480, 480, c) as e:
            e.distribute(A, x)
            for _ in range(3):
                e.multiply()
            y = e.collect()
        assert max_rel(y, golden[f"sq_480/{alg}/P1"]) <= TOL
    finally:
        c.destroy()


@pytest.mark.parametrize("ring", [1, 2, 8])
@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
def test_engine_exchange_overlap_keeps_each_multiply_own_y(alg, ring, monkeypatch):
    # The exchange of multiply i runs on its own stream beside the next multiplies' GEMVs, with
    # the partial y in a ring of `ring` buffers (1: exchange on the GEMV stream). Changing x
    # between back-to-back multiplies (no sync in between, across ring wrap-arounds) must still
    # leave exactly the last multiply's y on the root, and a collect in between must see its own
    # multiply's y.
    monkeypatch.setenv("MVG_ALWAYS_COLLECT", "1")
    monkeypatch.setenv("MVG_XRING", str(ring))
    c = mm.Comm.init_all([0])
    R, Cn = 2048, 4096
    A = oracle.synth(R, Cn, 42)
    xs = [oracle.synth(1, Cn, s)[0] for s in (11, 12, 13, 14)]
    want = [oracle.multiply(alg, A, x, 1) for x in xs]
    try:
        with mm.Multiplier(alg, R, Cn, c) as e:
            e.distribute(A, xs[0])
            e.multiply()
            assert max_rel(e.collect(), want[0]) <= TOL
            for x in xs[1:]:
                e.distribute(A, x)
                e.multiply()
                e.multiply()
            assert max_rel(e.collect(), want[-1]) <= TOL
            e.distribute(A, xs[1])
            for _ in range(5):
                e.multiply()
            e.sync()
            assert max_rel(e.collect(), want[1]) <= TOL
            for i in range(19):
                e.distribute(A, xs[i % 4])
                e.multiply()
            assert max_rel(e.collect(), want[18 % 4]) <= TOL
    finally:
        c.destroy()


def test_engine_rank_mode_world_of_one(golden):
    uid = mm.Comm.unique_id()
    c = mm.Comm.init_rank(uid, 1, 0, 0)
    try:
        A, x = case_inputs({"source": "fixture", "R": 4, "C": 8})
        with mm.Multiplier("colwise", 4, 8, c) as e:
            e.distribute(A, x)
            e.multiply()
            np.testing.assert_allclose(e.collect(), golden["fixture_4x8/colwise/P1"], rtol=TOL)
    finally:
        c.destroy()


def test_engine_shard_products_compose_to_golden_at_p_gt_1(golden, manifest):
    """Every rank's local product for P > 1, run on the GPU from the planner's shard, then
    combined by the exchange schedule's semantics, matches the reference's y at that P."""
    for case, alg, p in golden_runs(manifest):
        if p == 1:
            continue
        A, x = case_inputs(case)
        R, Cn = case["R"], case["C"]
        y = np.zeros(R)
        for r in range(p):
            s = mm.plan_shard(alg, R, Cn, p, r)
            blk = A[s.row_off:s.row_off + s.n_rows, s.col_off:s.col_off + s.n_cols]
            part = mm.multiply_std_rowwise(blk, x[s.col_off:s.col_off + s.n_cols])
            if alg == "colwise":
                y += part
            else:
                y[s.y_off:s.y_off + s.y_len] += part
        key = f"{case['name']}/{alg}/P{p}"
        assert max_rel(y, golden[key]) <= TOL, key


# ---------------------------------------------------------------- full BASELINE sizes
def _sampled_rows_check(e: "mm.Multiplier", R, Cn, y, rows):
    for r in rows:
        a = oracle.synth_block(int(r), 1, 0, Cn, Cn, 42)[0]
        xv = oracle.synth_block(0, 1, 0, Cn, Cn, 4242)[0]
        want = oracle.multiply_std_rowwise(a[None, :], xv)[0]
        assert abs(y[r] - want) <= TOL * abs(want), (R, Cn, r)


@pytest.mark.parametrize("alg,R,Cn", [
    ("rowwise", 16384, 16384),     # config 2
    ("rowwise", 524288, 512),      # config 5's per-GPU shard (4,194,304 x 512 over 8 GPUs)
    ("colwise", 65536, 65536),     # config 3 at G = 1 (32 GiB on the device)
    ("blockwise", 65536, 32768),   # config 4's per-GPU block (131072^2 on a 2 x 4 grid)
    ("rowwise", 4194304, 512),     # config 5 whole on one GPU (16 GiB)
    ("blockwise", 131072, 131072),  # config 4 whole on one GPU (1 x 1 grid, 128 GiB)
])
def test_full_size_sampled_rows_and_properties(comm1, alg, R, Cn):
    rng = np.random.default_rng(7)
    rows = np.unique(np.concatenate([[0, 1, R // 2, R - 1], rng.integers(0, R, 60)]))
    with mm.Multiplier(alg, R, Cn, comm1) as e:
        e.fill_synth()
        e.multiply()
        y1 = e.collect()
        e.multiply()
        y2 = e.collect()
    np.testing.assert_array_equal(y1, y2)  # deterministic run to run
    assert np.all(np.isfinite(y1))
    _sampled_rows_check(e, R, Cn, y1, rows)
    # checksum: sum(y) = sum_j x_j * colsum_j is too costly here; instead every y_i lies in
    # [0, C * 0.9999^2] for inputs in [0, 0.9999]
    assert y1.min() >= 0 and y1.max() <= Cn * 0.9999 * 0.9999


def _oracle_y_by_row_blocks(R, Cn, block_bytes=256 << 20):
    """The oracle's y = multiply_std_rowwise(A, x) of the synthetic A (seed 42) and x (4242),
    generated and summed in row blocks on the host's allowed CPUs (ctypes releases the GIL), so
    config 4's 128 GiB A is never held whole."""
    from concurrent.futures import ThreadPoolExecutor

    x = oracle.synth(1, Cn, 4242)[0]
    y = np.empty(R)
    rows = max(1, block_bytes // (8 * Cn))

    def block(r0):
        nr = min(rows, R - r0)
        y[r0:r0 + nr] = oracle.multiply_std_rowwise(oracle.synth_block(r0, nr, 0, Cn, Cn, 42), x)

    with ThreadPoolExecutor(max_workers=max(1, min(16, len(os.sched_getaffinity(0))))) as ex:
        list(ex.map(block, range(0, R, rows)))
    return y


@pytest.mark.parametrize("alg,R,Cn", [
    ("rowwise", 16384, 16384),     # config 2
    ("rowwise", 524288, 512),      # config 5's per-GPU shard
    ("colwise", 65536, 8192),      # config 3's per-GPU strip shape (65536^2 over 8 GPUs)
    ("blockwise", 65536, 32768),   # config 4's per-GPU block (131072^2 on a 2 x 4 grid)
    ("rowwise", 4194304, 512),     # config 5 whole on one GPU (16 GiB)
    ("colwise", 65536, 65536),     # config 3 whole on one GPU (32 GiB)
    ("blockwise", 131072, 131072),  # config 4 whole on one GPU (1 x 1 grid, 128 GiB)
])
def test_full_size_whole_y_against_oracle(comm1, alg, R, Cn):
    """Every row of y at the BASELINE configs' per-GPU shapes against the oracle's sequential
    sums: tree mode within TOL, exact mode bit for bit — on the row-major kernels (first
    multiply) and on the engine's column-panel copy where it builds one (second multiply). At
    P = 1 each multiplier's y is multiply_std_rowwise's: a one-strip column split scales in place
    and sums from 0.0 (multiplier_colwise.c:107-122), a 1 x 1 grid adds its one partial to 0
    (multiplier_blockwise.c:206) — the golden vectors pin that at P = 1."""
    want = _oracle_y_by_row_blocks(R, Cn)
    with mm.Multiplier(alg, R, Cn, comm1) as e:
        e.fill_synth()
        e.multiply()
        y = e.collect()
        e.set_exact(True)
        e.multiply()
        y_rm = e.collect()
        e.multiply()
        y_2 = e.collect()
    assert max_rel(y, want) <= TOL
    np.testing.assert_array_equal(y_rm, want)
    np.testing.assert_array_equal(y_2, want)


def test_scaling_x_by_two_is_exact():
    # size-independent property: the kernel is linear and scaling by 2 is exact in fp64,
    # so y(A, 2x) == 2 * y(A, x) bit for bit
    m, k = 8192, 8192
    dA, dx, dy = mm.DeviceBuffer(m * k), mm.DeviceBuffer(k), mm.DeviceBuffer(m)
    _lib.check(_lib.lib.mvg_synth_fill_device(dA.ptr, k, m, k, 0, 0, k, 42, None), "fill")
    x = oracle.synth(1, k, 4242)[0]
    dx.upload(x)
    mm.gemv(dA.ptr, k, dx.ptr, dy.ptr, m, k)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    y = dy.download()
    dx.upload(2.0 * x)
    mm.gemv(dA.ptr, k, dx.ptr, dy.ptr, m, k)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    np.testing.assert_array_equal(dy.download(), 2.0 * y)


def test_text_input_end_to_end(tmp_path, comm1):
    # the executables' path: text files in the reference format -> loader -> engine -> y
    R, Cn = 96, 160
    mm.write_matr_synth(str(tmp_path / f"matrix_{R}_{Cn}.txt"), R, Cn, 42)
    mm.write_matr_synth(str(tmp_path / f"vector_{Cn}.txt"), 1, Cn, 4242)
    A, x = mm.load_matr(R, Cn, str(tmp_path)), mm.load_vec(Cn, str(tmp_path))
    for alg in ("rowwise", "colwise", "blockwise"):
        with mm.Multiplier(alg, R, Cn, comm1) as e:
            e.distribute(A, x)
            e.multiply()
            assert max_rel(e.collect(), oracle.multiply(alg, A, x, 1)) <= TOL


def test_engine_distribute_shared_and_kernel_timing(comm1, golden):
    A, x = oracle.synth(480, 480, 42), oracle.synth(1, 480, 4242)[0]
    for alg in ("rowwise", "colwise", "blockwise"):
        with mm.Multiplier(alg, 480, 480, comm1) as e:
            e.distribute_shared(A, x)
            e.kernel_timing(2)
            for _ in range(6):
                e.multiply()
            kt = e.kernel_ms()
            e.kernel_timing(0)
            assert kt.launches == 3 and kt.avg_ms > 0
            assert max_rel(e.collect(), golden[f"sq_480/{alg}/P1"]) <= TOL


def test_engine_multiply_before_inputs_is_state_error(comm1):
    with mm.Multiplier("rowwise", 8, 8, comm1) as e:
        with pytest.raises(_lib.MvgError) as err:
            e.multiply()
        assert err.value.code == _lib.MVG_E_STATE


@pytest.mark.parametrize("m,k,nv", [(257, 1000, 1), (64, 16384, 2), (130, 4096, 3), (33, 20000, 5), (9, 512, 8),
                                    (100, 3000, 11), (50, 1001, 4),
                                    # the automatic DMA forms, with row and tile tails
                                    (8195, 1030, 8), (8200, 1290, 3), (8197, 6150, 2), (4099, 8194, 6),
                                    (8192, 1024, 16), (8203, 1058, 13), (8193, 2050, 25)])
def test_multi_vector_gemv(m, k, nv):
    A = oracle.synth(m, k, 42)
    X = oracle.synth(nv, k, 4242).T  # k x nv
    Y = mm.multiply_multi(A, X)
    assert Y.shape == (m, nv)
    for v in range(nv):
        assert max_rel(Y[:, v], oracle.multiply_std_rowwise(A, np.ascontiguousarray(X[:, v]))) <= TOL, v


@pytest.mark.parametrize("m,k,nv", [(257, 1000, 2), (130, 4226, 4), (33, 6002, 8), (1000, 512, 3), (77, 256, 8),
                                    (9, 130, 5), (4099, 64, 2)])
def test_multi_vector_every_variant(m, k, nv):
    """Every mvg_gemv_multi kernel variant, with row and column tails (rows not a multiple of a
    block's rows, K not a multiple of a chunk), against the oracle per vector; columns of Y past
    nv are never written."""
    from matvec_mpi_multiplier_amd._lib import check, lib

    A = oracle.synth(m, k, 42)
    X = oracle.synth(nv, k, 4242)  # nv x k: vector v contiguous (column-major k x nv)
    want = [oracle.multiply_std_rowwise(A, np.ascontiguousarray(X[v])) for v in range(nv)]
    dA, dX = mm.DeviceBuffer(m * k).upload(A), mm.DeviceBuffer(nv * k).upload(X)
    dY = mm.DeviceBuffer(m * 8)
    try:
        for var in range(1, lib.mvg_gemv_multi_variant_count()):
            name = lib.mvg_gemv_multi_variant_name(var).decode()
            dY.upload(np.full(m * 8, np.nan))
            check(lib.mvg_gemv_multi_variant(dA.ptr, k, dX.ptr, k, dY.ptr, m, m, k, nv, var, None), name)
            check(lib.mvg_stream_sync(None), "sync")
            Y = dY.download(m * 8).reshape(8, m)
            for v in range(nv):
                assert max_rel(Y[v], want[v]) <= TOL, (name, v)
            assert np.isnan(Y[nv:]).all(), name
    finally:
        for b in (dA, dX, dY):
            b.free()


@pytest.mark.parametrize("m,k,nv", [(257, 1000, 16), (33, 6002, 11), (130, 4226, 9), (77, 256, 16), (9, 130, 12),
                                    (4099, 64, 16), (1000, 512, 3)])
def test_multi_vector_16_per_pass_every_variant(m, k, nv):
    """The 16-vector matrix-core variants (gemv_mdma16) on every shape class: row tails, tile
    tails (K not a multiple of a tile), K shorter than a tile, vectors past nv never written."""
    from matvec_mpi_multiplier_amd._lib import check, lib

    A = oracle.synth(m, k, 42)
    X = oracle.synth(nv, k, 4242)
    want = [oracle.multiply_std_rowwise(A, np.ascontiguousarray(X[v])) for v in range(nv)]
    dA, dX = mm.DeviceBuffer(m * k).upload(A), mm.DeviceBuffer(nv * k).upload(X)
    dY = mm.DeviceBuffer(m * 16)
    try:
        names = [lib.mvg_gemv_multi_variant_name(v).decode() for v in range(lib.mvg_gemv_multi_variant_count())]
        m16 = [v for v, n in enumerate(names) if n.startswith("m16_")]
        assert m16
        for var in m16:
            dY.upload(np.full(m * 16, np.nan))
            check(lib.mvg_gemv_multi_variant(dA.ptr, k, dX.ptr, k, dY.ptr, m, m, k, nv, var, None), names[var])
            check(lib.mvg_stream_sync(None), "sync")
            Y = dY.download(m * 16).reshape(16, m)
            for v in range(nv):
                assert max_rel(Y[v], want[v]) <= TOL, (names[var], v)
            assert np.isnan(Y[nv:]).all(), names[var]
    finally:
        for b in (dA, dX, dY):
            b.free()


def test_distribute_shared_from_dev_shm(comm1, golden, tmp_path):
    """bench.py's N > 1 'shared' end-to-end path at world size 1: A in a /dev/shm segment,
    pinned with hipHostRegister, pulled by the GPU, y vs the reference's golden y."""
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd.hostshare import SharedHostMatrix

    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        sh = SharedHostMatrix.create(480, 480, 42, f"gputest_{os.getpid()}", margin=0)
        assert sh is not None
        A = sh.array
        x = oracle.synth(1, 480, 4242)[0]
        assert _lib.lib.mvg_host_register(A.ctypes.data, A.nbytes) == 0
        with mm.Multiplier("colwise", 480, 480, comm1) as e:
            e.distribute_shared(A, x)
            e.multiply()
            y = e.collect()
            e._keep = None
        _lib.lib.mvg_host_unregister(A.ctypes.data)
        del A
        sh.close()
        assert max_rel(y, golden["sq_480/colwise/P1"]) <= TOL
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_device_numa_node_and_first_touch():
    """The GPU's NUMA node comes from its PCI address (sysfs); first touch near it zeroes."""
    import ctypes as C

    node = C.c_int(-2)
    assert _lib.lib.mvg_device_numa_node(0, C.byref(node)) == 0
    assert node.value >= -1
    a = np.full(10_000_000, 1.0)
    assert _lib.lib.mvg_host_first_touch(a.ctypes.data, a.nbytes, 0) == 0 and not a.any()


# ---------------------------------------------------------------- chunked distribution overlap
@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
def test_writes_right_after_a_chunked_distribution(comm1, alg):
    """drain_chunks (csrc/engine.cpp): a chunked distribution's copies may still be running on the
    copy stream when the next write of the shard is queued. A second distribute, or fill_synth,
    with no multiply and no sync in between must land after them, and the next multiply must read
    the whole new shard."""
    R, C = 1000, 768
    A1, A2 = oracle.synth(R, C, 42), oracle.synth(R, C, 7)
    x1, x2 = oracle.synth(1, C, 4242)[0], oracle.synth(1, C, 99)[0]
    for exact in (False, True):
        with mm.Multiplier(alg, R, C, comm1, exact=exact) as e:
            e.set_overlap(5)
            ys = []
            e.distribute(A1, x1)
            e.distribute(A2, x2)  # chunked copies of A1 still queued: A2 must win
            e.multiply()
            ys.append(e.collect())
            e.distribute(A2, x2)
            e.fill_synth()  # seeds 42 / 4242: A1, x1 on the device, after A2's chunks
            e.multiply()
            ys.append(e.collect())
            e.distribute(A2, x1)
            e.set_overlap(0)
            e.distribute(A1, x2)  # a whole-shard write while the chunks are still pending
            e.multiply()
            ys.append(e.collect())
        for y, (A, x) in zip(ys, ((A2, x2), (A1, x1), (A1, x2))):
            want = oracle.multiply(alg, A, x, 1)
            if exact:
                assert np.array_equal(y, want), alg
            else:
                assert max_rel(y, want) <= TOL, alg


@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
@pytest.mark.parametrize("chunks", [2, 7])
def test_overlapped_distribution_gives_the_same_y(comm1, alg, chunks):
    """mvg_engine_set_overlap: the shard goes over in row chunks and each chunk's GEMV runs behind
    its copy. Back-to-back distribute/multiply cycles with different inputs and no sync in
    between (the copies must wait for the GEMV still reading the shard), tree and exact mode."""
    R, C = 1000, 768
    A1, A2 = oracle.synth(R, C, 42), oracle.synth(R, C, 7)
    x1, x2 = oracle.synth(1, C, 4242)[0], oracle.synth(1, C, 99)[0]
    for exact in (False, True):
        with mm.Multiplier(alg, R, C, comm1, exact=exact) as e:
            e.set_overlap(chunks)
            ys = []
            for A, x in ((A1, x1), (A2, x2), (A1, x2)):
                e.distribute(A, x)
                e.multiply()
                ys.append(e.collect())
            # no collect (no sync) between: the second copies must wait for the first GEMV
            e.distribute(A1, x1)
            e.multiply()
            e.distribute(A2, x2)
            e.multiply()
            ys.append(e.collect())
            e.set_overlap(0)
            e.distribute(A2, x1)
            e.multiply()
            ys.append(e.collect())
        for y, (A, x) in zip(ys, ((A1, x1), (A2, x2), (A1, x2), (A2, x2), (A2, x1))):
            want = oracle.multiply(alg, A, x, 1)
            if exact:
                assert np.array_equal(y, want), (alg, chunks)
            else:
                assert max_rel(y, want) <= TOL, (alg, chunks)


@pytest.mark.gpu
def test_library_and_pytorch_share_the_device_in_any_order():
    """PyTorch's wheel bundles its own HIP + HSA runtimes; two HSA runtimes in one process cannot
    both open the GPU (profiles/r05/torch_order/library_first.err). The package imports PyTorch
    before loading the library, so both runtimes work whichever touches the device first."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, {repo!r})\n"
            "from matvec_mpi_multiplier_amd import multiplier as mm\n"
            "import numpy as np, torch\n"
            "{first}\n"
            "A = np.arange(64 * 48, dtype=np.float64).reshape(64, 48) / 7; x = np.linspace(0, 1, 48)\n"
            "y = mm.multiply_std_rowwise(A, x)\n"
            "{second}\n"
            "assert np.allclose(y, A @ x, rtol=1e-13, atol=0)\n"
            "print('ok', float(t.sum()))\n")
    torch_op = "torch.cuda.set_device(0); t = torch.ones(1000, device='cuda:0', dtype=torch.float64); torch.cuda.synchronize()"
    for first, second in ((torch_op, ""), ("", torch_op)):
        r = subprocess.run([sys.executable, "-c", code.format(repo=REPO_ROOT, first=first, second=second)],
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0 and r.stdout.startswith("ok 1000.0"), r.stderr[-2000:]


def test_span_kernel_timing_agrees_with_per_launch_events(comm1):
    """mvg_engine_kernel_timing(-1): one event pair from the first GEMV of the span to the next
    sync, averaged over its multiplies; it must agree with events on every launch (config 2's
    shape, the bench's headline kernel) and reset at kernel_timing()."""
    R = C = 16384
    with mm.Multiplier("rowwise", R, C, comm1) as e:
        e.fill_synth()
        for _ in range(30):
            e.multiply()
        e.kernel_timing(1)
        for _ in range(30):
            e.multiply()
        per_launch = e.kernel_ms()
        e.kernel_timing(-1)
        for _ in range(30):
            e.multiply()
        e.sync()
        for _ in range(20):  # a second span after the sync adds up with the first
            e.multiply()
        span = e.kernel_ms()
        e.kernel_timing(0)
    assert per_launch.launches == 30 and span.launches == 50
    assert 0.2 < span.avg_ms < 0.5 and abs(span.avg_ms - per_launch.avg_ms) <= 0.05 * per_launch.avg_ms, (span, per_launch)


def test_span_kernel_timing_drops_a_span_that_holds_other_writes(comm1):
    """A span that also holds a write of the shard — a synthetic fill, a distribution, exact
    mode's panel relayout after the span's first GEMV — no longer times GEMVs alone: it adds
    neither launches nor time; the spans around it still count."""
    R = C = 8192
    A = oracle.synth(R, C, 42)
    x = oracle.synth(1, C, 4242)[0]
    with mm.Multiplier("rowwise", R, C, comm1) as e:
        e.fill_synth()
        e.kernel_timing(-1)
        for _ in range(5):
            e.multiply()
        e.sync()  # a clean span: 5 launches
        e.multiply()
        e.fill_synth()  # inside the open span
        e.multiply()
        e.sync()
        e.multiply()
        e.distribute(A, x)  # inside the open span
        e.multiply()
        assert e.kernel_ms().launches == 5
        e.set_exact(True)
        e.distribute(A, x)
        e.multiply()
        e.sync()  # exact, first multiply of a distribution: row-major kernels, no relayout (counted)
        n = e.kernel_ms().launches
        e.multiply()  # a span opened on the second multiply: the relayout runs before its first event
        e.multiply()
        e.sync()
        n2 = e.kernel_ms().launches
        assert e.exact_panel_width() == 256  # this shape runs exact mode on the column-panel copy
        e.distribute(A, x)  # panels stale again
        e.multiply()  # opens the span (row-major exact kernels)
        e.multiply()  # the relayout runs after the span's first event: the span is dropped
        e.sync()
        n3 = e.kernel_ms().launches
        e.set_exact(False)
        e.kernel_timing(0)
    assert n == 6 and n2 == 8 and n3 == 8
