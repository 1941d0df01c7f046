"""Bit-exact mode (mvg_gemv_exact, mvg_engine_set_exact): y identical to the reference's, not
just within 1e-12.

The reference's row sum is a sequential chain of rounded multiplies and rounded adds
(src/matr_utils.c:87-93), its column split combines strips with MPICH's binomial MPI_Reduce
(colwise.c:124) and its block split adds the grid row's partials into a zeroed y
(blockwise.c:150-207). The exact kernels reproduce all of it, so every comparison here is
np.array_equal — against the oracle (the pinned C restatement) on the same inputs, and against
the golden y the real reference wrote (tests/golden), wherever the reference is deterministic
(block split with more than two grid columns adds in message-arrival order; there the check is
against the oracle's rank order, and within the tolerance against the reference).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import case_inputs, golden_runs, max_rel
from matvec_mpi_multiplier_amd import _lib
from matvec_mpi_multiplier_amd import multiplier as mm
from oracle import oracle

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1), (1, 2), (3, 5), (4, 8), (5, 7), (63, 129), (64, 128), (65, 127), (257, 1000), (1000, 257),
          (33, 4096), (7, 20001), (2049, 512), (100, 1), (100, 2), (100, 3), (130, 16388), (3, 65538),
          (200, 96), (129, 32), (64, 33), (700, 2080)]


def signed(A, seed):
    """Mixed-sign inputs: bit-exactness does not depend on the data being non-negative."""
    rng = np.random.default_rng(seed)
    return A * rng.choice([-1.0, 1.0], size=A.shape)


def needs_16b(name):
    """16-B loads (LDS-DMA or plain): 16-B aligned A and x and an even lda; `hop8_*` (8-B loads),
    `seq_scalar` and `auto` take anything."""
    return name.startswith(("seq_r", "seqx_", "hop_"))


def xl_k_limited(name):
    """`hopxl_*` stage all of x in LDS: k <= 8192 (64 KiB), refused above."""
    return name.startswith("hopxl_")


def exact_variants():
    lib = _lib.lib
    return [(v, lib.mvg_gemv_exact_variant_name(v).decode()) for v in range(lib.mvg_gemv_exact_variant_count())]


@pytest.mark.parametrize("m,k", SHAPES)
def test_gemv_exact_every_variant_is_the_reference_sum(m, k):
    A = signed(oracle.synth(m, k, 42), m * 7 + k)
    x = signed(oracle.synth(1, k, 4242)[0], k)
    want = oracle.multiply_std_rowwise(A, x)
    for v, name in exact_variants():
        if (needs_16b(name) and k % 2) or (xl_k_limited(name) and k > 8192):  # forms that refuse the shape
            with pytest.raises(_lib.MvgError):
                mm.multiply_std_rowwise(A, x, variant=v, exact=True)
            continue
        y = mm.multiply_std_rowwise(A, x, variant=v, exact=True)
        assert np.array_equal(y, want), (name, m, k, max_rel(y, want))


def test_gemv_exact_hop_segment_edges():
    # the chain-hopping forms (hop_l<L>_w<W>_u<U>, hop8_* with 8-B loads): a segment is S = L*W columns and U segments
    # are in flight; after an odd number of segments the chain ends in lane L-1, after an even
    # number in lane 0, so every variant is run with odd and even segment counts, with and
    # without leftover segments (nseg % U), a column tail, no whole segment at all, and a
    # last wave with rows to spare
    for v, name in exact_variants():
        if not name.startswith("hop"):
            continue
        L, W, U = (int(part[1:]) for part in name.split("_")[1:4])
        nw = int(name.split("_n")[-1]) if xl_k_limited(name) else 1  # waves per workgroup
        S = L * W
        m = 3 * nw * (64 // L) + 1
        ks = [S - 2, S, 3 * S + 2, (U + 1) * S, (U + 1) * S + 2, (U + 2) * S, 2 * U * S, 2 * U * S + 2,
              (3 * U - 1) * S]
        if not needs_16b(name):  # odd widths too: every other row starts 8 bytes off a 16-B boundary
            ks += [k + 1 for k in ks]
        for k in ks:
            A = signed(oracle.synth(m, k, 42), k)
            x = signed(oracle.synth(1, k, 4242)[0], k + 1)
            y = mm.multiply_std_rowwise(A, x, variant=v, exact=True)
            assert np.array_equal(y, oracle.multiply_std_rowwise(A, x)), (name, m, k)


def test_gemv_exact_rows_beyond_lds_offsets():
    # lda >= 2^23 doubles: past the LDS forms' 32-bit per-lane offsets; the dispatch takes a
    # chain-hopping form (64-bit addressing), which must still be the reference's sum
    m, k = 3, (1 << 23) + 34
    A = signed(oracle.synth(m, k, 42), 5)
    x = signed(oracle.synth(1, k, 4242)[0], 6)
    names = dict(exact_variants())
    assert names[_lib.lib.mvg_gemv_exact_auto_variant(k, m, k)].startswith("hop")
    assert np.array_equal(mm.multiply_std_rowwise(A, x, exact=True), oracle.multiply_std_rowwise(A, x))
    lds = next(v for v, name in exact_variants() if name.startswith("seqx_"))
    with pytest.raises(_lib.MvgError):
        mm.multiply_std_rowwise(A, x, variant=lds, exact=True)


def test_gemv_exact_padded_lda_misaligned_and_k_zero():
    m, k, lda = 130, 300, 512
    full = oracle.synth(m, lda, 42)
    x = oracle.synth(1, k + 1, 4242)[0]
    dA, dx, dy = mm.DeviceBuffer(m * lda).upload(full), mm.DeviceBuffer(k + 1).upload(x), mm.DeviceBuffer(m)
    want = oracle.multiply_std_rowwise(full[:, :k], x[:k])
    for v, name in exact_variants():
        mm.gemv(dA.ptr, lda, dx.ptr, dy.ptr, m, k, None, v, exact=True)
        _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
        assert np.array_equal(dy.download(), want), name
    # A and x 8 bytes off a 16-B boundary: the automatic choice takes the 8-B path
    want = oracle.multiply_std_rowwise(full[:, 1:k + 1], x[1:k + 1])
    mm.gemv(dA.ptr + 8, lda, dx.ptr + 8, dy.ptr, m, k, None, 0, exact=True)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    assert np.array_equal(dy.download(), want)
    with pytest.raises(_lib.MvgError):  # a 16-B variant refuses the misaligned operands
        mm.gemv(dA.ptr + 8, lda, dx.ptr + 8, dy.ptr, m, k, None, 2, exact=True)
    dy.upload(np.full(m, 7.0))
    mm.gemv(dA.ptr, lda, dx.ptr, dy.ptr, m, 0, None, 0, exact=True)
    _lib.check(_lib.lib.mvg_stream_sync(None), "sync")
    assert np.array_equal(dy.download(), np.zeros(m))  # the reference's `sum = 0`


def test_gemv_exact_reference_fixture_digits():
    # data/matrix_4_8.txt x data/vector_8.txt: the reference's y printed with %.17g
    from conftest import GOLDEN_DIR

    A = np.loadtxt(os.path.join(GOLDEN_DIR, "matrix_4_8.txt")).reshape(4, 8)
    x = np.loadtxt(os.path.join(GOLDEN_DIR, "vector_8.txt")).reshape(8)
    y = mm.multiply_std_rowwise(A, x, exact=True)
    assert ["%.17g" % v for v in y] == ["222.19999999999999", "196.55000000000001", "191.56999999999999",
                                        "232.90000000000001"]


@pytest.mark.parametrize("m,k", [(16384, 16384), (4096, 65536), (262144, 512)])
def test_gemv_exact_full_width_rows_sampled(m, k):
    """Large shapes on device-resident synthetic data: sampled rows against the oracle, bit for
    bit, and run-to-run identity."""
    s = None
    dA, dx, dy = mm.DeviceBuffer(m * k), mm.DeviceBuffer(k), mm.DeviceBuffer(m)
    _lib.check(_lib.lib.mvg_synth_fill_device(dA.ptr, k, m, k, 0, 0, k, 42, s), "fill")
    _lib.check(_lib.lib.mvg_synth_fill_device(dx.ptr, k, 1, k, 0, 0, k, 4242, s), "fill")
    mm.gemv(dA.ptr, k, dx.ptr, dy.ptr, m, k, s, 0, exact=True)
    _lib.check(_lib.lib.mvg_stream_sync(s), "sync")
    y = dy.download()
    rows = np.unique(np.r_[0, 1, 63, 64, m // 2, m - 2, m - 1, np.random.default_rng(0).integers(0, m, 24)])
    x = oracle.synth(1, k, 4242)[0]
    for r in rows:
        Ar = oracle.synth_block(int(r), 1, 0, k, k, 42)
        assert oracle.multiply_std_rowwise(Ar, x)[0] == y[r], r
    mm.gemv(dA.ptr, k, dx.ptr, dy.ptr, m, k, s, 0, exact=True)
    _lib.check(_lib.lib.mvg_stream_sync(s), "sync")
    assert np.array_equal(dy.download(), y)


# ---------------------------------------------------------------- the engine in exact mode
@pytest.fixture(scope="module")
def comm1():
    c = mm.Comm.init_all([0])
    yield c
    c.destroy()


def test_engine_exact_p1_equals_every_golden_p1(comm1, golden, manifest):
    for case, alg, p in golden_runs(manifest):
        if p != 1 or case["R"] * case["C"] > 50_000_000:
            continue
        A, x = case_inputs(case)
        with mm.Multiplier(alg, case["R"], case["C"], comm1, exact=True) as e:
            assert e.exact
            e.distribute(A, x)
            e.multiply()
            y = e.collect()
        assert np.array_equal(y, golden[f"{case['name']}/{alg}/P1"]), (case["name"], alg)


@pytest.mark.parametrize("alg", ["rowwise", "colwise", "blockwise"])
def test_engine_exact_forced_collectives_p1(alg, monkeypatch, golden):
    # the exact exchange (ncclGather of the partials + the combine kernel on rank 0) at world
    # size 1, with the ring of partial buffers wrapping around
    monkeypatch.setenv("MVG_ALWAYS_COLLECT", "1")
    monkeypatch.setenv("MVG_EXACT", "1")
    A, x = oracle.synth(480, 480, 42), oracle.synth(1, 480, 4242)[0]
    c = mm.Comm.init_all([0])
    try:
        with mm.Multiplier(alg, 480, 480, c) as e:
            assert e.exact
            e.distribute(A, x)
            for _ in range(11):
                e.multiply()
            y = e.collect()
    finally:
        c.destroy()
    assert np.array_equal(y, golden[f"sq_480/{alg}/P1"])


def test_engine_exact_shard_products_and_combines_at_p_gt_1(golden, manifest):
    """P > 1 on one GPU: every rank's shard product with mvg_gemv_exact, combined in the
    reference's order (the engine's combine kernels' order, restated on the host) — against the
    golden y of the real reference at the same P, bit for bit where the reference is
    deterministic."""
    for case, alg, p in golden_runs(manifest):
        if p == 1 or case["R"] * case["C"] > 50_000_000:
            continue
        A, x = case_inputs(case)
        R, C = case["R"], case["C"]
        parts = []
        for r in range(p):
            sh = mm.plan_shard(alg, R, C, p, r)
            blk = np.ascontiguousarray(A[sh.row_off:sh.row_off + sh.n_rows, sh.col_off:sh.col_off + sh.n_cols])
            parts.append(mm.multiply_std_rowwise(blk, x[sh.col_off:sh.col_off + sh.n_cols], exact=True))
        if alg == "rowwise":
            y = np.concatenate(parts)
        elif alg == "colwise":  # MPICH's MPI_Reduce order (the engine's combine_mpich)
            y = oracle.mpich_reduce(parts)
        else:
            gr, gc = mm.get_2_most_closest_multipliers(p)
            y = np.zeros(R)
            lr = R // gr
            for r in range(p):
                y[(r // gc) * lr:(r // gc + 1) * lr] += parts[r]
        key = f"{case['name']}/{alg}/P{p}"
        if alg == "blockwise" and mm.get_2_most_closest_multipliers(p)[1] > 2:
            assert np.array_equal(y, oracle.multiply(alg, A, x, p)), key
            assert max_rel(y, golden[key]) <= 1e-12, key
        else:
            assert np.array_equal(y, golden[key]), key


def test_multiply_std_rowwise_host_entry_point():
    # mvg_multiply_std_rowwise: the reference's in-process call (matr_utils.h:4-10) on host
    # pointers — bit for bit with exact=1, within the bar otherwise; the per-thread device
    # buffers grow across calls of rising size and are released by the all-null call
    import ctypes as C

    lib = _lib.lib

    def call(A, x, exact):
        y = np.full(A.shape[0], np.nan)
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        _lib.check(lib.mvg_multiply_std_rowwise(ptr(A), ptr(x), A.shape[0], A.shape[1], ptr(y), exact), "call")
        return y

    from conftest import GOLDEN_DIR

    A = np.ascontiguousarray(np.loadtxt(os.path.join(GOLDEN_DIR, "matrix_4_8.txt")).reshape(4, 8))
    x = np.ascontiguousarray(np.loadtxt(os.path.join(GOLDEN_DIR, "vector_8.txt")).reshape(8))
    assert ["%.17g" % v for v in call(A, x, 1)] == ["222.19999999999999", "196.55000000000001",
                                                  "191.56999999999999", "232.90000000000001"]
    for m, k in [(3, 5), (7, 20001), (130, 16388), (4200, 4200), (1200, 6000)]:
        # the reference's own inputs (non-negative: the 1e-12 relative bar applies row by row)
        A, x = oracle.synth(m, k, 42), oracle.synth(1, k, 4242)[0]
        want = oracle.multiply_std_rowwise(A, x)
        assert max_rel(call(A, x, 0), want) <= 1e-12, (m, k)
        # mixed signs: bit for bit still
        A, x = np.ascontiguousarray(signed(A, k)), np.ascontiguousarray(signed(x, m))
        assert np.array_equal(call(A, x, 1), oracle.multiply_std_rowwise(A, x)), (m, k)
    assert np.array_equal(call(np.zeros((5, 0)), np.zeros(0), 1), np.zeros(5))  # sum = 0
    _lib.check(lib.mvg_multiply_std_rowwise(None, None, 0, 0, None, 0), "release")
    with pytest.raises(_lib.MvgError):
        _lib.check(lib.mvg_multiply_std_rowwise(None, None, 3, 3, None, 1), "null")


# ---------------------------------------------------------------- column-panel layout
def panel_variants():
    lib = _lib.lib
    return [(v, lib.mvg_gemv_exact_panel_variant_name(v).decode())
            for v in range(lib.mvg_gemv_exact_panel_variant_count())]


def panels_of(A, P):
    """Host restatement of the panel layout (mvg_panel_relayout): panel p = columns
    [pP, pP + P) of every row, rows P apart, panels m*P apart, the last one padded to P."""
    m, k = A.shape
    npan = -(-k // P)
    out = np.zeros((npan, m, P))
    for p in range(npan):
        w = min(P, k - p * P)
        out[p, :, :w] = A[:, p * P:p * P + w]
    return out


@pytest.mark.parametrize("m,k", [(1, 16), (9, 2048), (65, 4096 + 2), (130, 257), (1000, 1536), (61, 16388),
                                 (640, 8191), (3, 1), (8, 0)])
def test_gemv_exact_panels_every_variant_is_the_reference_sum(m, k):
    # the relayout kernel against the host restatement of the layout, then every panel variant
    # and panel width over it against the oracle, bit for bit (mixed signs; column tails of every
    # length; rows past the last whole wave; a padded row-major source with lda > k)
    lib = _lib.lib
    lda = k + 3
    A = signed(oracle.synth(m, lda, 42), m + k)
    x = signed(oracle.synth(1, k, 4242)[0], k + 1) if k else np.zeros(1)
    want = oracle.multiply_std_rowwise(np.ascontiguousarray(A[:, :k]), x[:k])
    dA, dx, dy = mm.DeviceBuffer(m * lda).upload(A), mm.DeviceBuffer(max(k, 1)).upload(x), mm.DeviceBuffer(m)
    for P in (16, 32, 256):
        npan = max(-(-k // P), 1)
        dAp = mm.DeviceBuffer(npan * m * P).upload(np.zeros(npan * m * P))
        _lib.check(lib.mvg_panel_relayout(dA.ptr, lda, m, k, dAp.ptr, m * P, P, None), "relayout")
        _lib.check(lib.mvg_stream_sync(None), "sync")
        if k:
            assert np.array_equal(dAp.download().reshape(npan, m, P), panels_of(A[:, :k], P)), P
        for v, name in panel_variants():
            seg = 32 if name.startswith("panel_l16") else 16
            rc = lib.mvg_gemv_exact_panels(dAp.ptr, m * P, P, dx.ptr, dy.ptr, m, k, v, None)
            if P % seg:
                assert rc != 0, (name, P)
                continue
            _lib.check(rc, name)
            _lib.check(lib.mvg_stream_sync(None), "sync")
            assert np.array_equal(dy.download(), want), (name, P, m, k)
        dAp.free()


def test_gemv_exact_panels_row_ranges_and_refusals():
    # the engine's chunked distribution relays out and multiplies row ranges (d_A + r0*lda,
    # d_Ap + r0*P, the whole shard's pstride): the pieces must give the whole y
    lib = _lib.lib
    m, k, P = 3001, 5000, 256
    A = signed(oracle.synth(m, k, 42), 3)
    x = signed(oracle.synth(1, k, 4242)[0], 4)
    want = oracle.multiply_std_rowwise(A, x)
    npan = -(-k // P)
    dA, dx, dy = mm.DeviceBuffer(m * k).upload(A), mm.DeviceBuffer(k).upload(x), mm.DeviceBuffer(m)
    dAp = mm.DeviceBuffer(npan * m * P)
    for r0, r1 in [(0, 1000), (1000, 1001), (1001, 2999), (2999, 3001)]:
        _lib.check(lib.mvg_panel_relayout(dA.ptr + 8 * r0 * k, k, r1 - r0, k, dAp.ptr + 8 * r0 * P, m * P, P, None), "rl")
        _lib.check(lib.mvg_gemv_exact_panels(dAp.ptr + 8 * r0 * P, m * P, P, dx.ptr, dy.ptr + 8 * r0, r1 - r0, k, 0,
                                             None), "gemv")
    _lib.check(lib.mvg_stream_sync(None), "sync")
    assert np.array_equal(dy.download(), want)
    assert lib.mvg_gemv_exact_panels(dAp.ptr, m * P, 96, dx.ptr, dy.ptr, m, k, 0, None) != 0  # P not 2^n
    assert lib.mvg_gemv_exact_panels(dAp.ptr, m * P, P, dx.ptr + 8, dy.ptr, m, k, 0, None) != 0  # x off 16 B
    assert lib.mvg_gemv_exact_panels(dAp.ptr, m * P - 1, P, dx.ptr, dy.ptr, m, k, 0, None) != 0  # pstride
    assert lib.mvg_panel_relayout(dA.ptr, k - 1, m, k, dAp.ptr, m * P, P, None) != 0  # lda < k


@pytest.mark.parametrize("alg", ["rowwise", "colwise"])
@pytest.mark.parametrize("overlap", [0, 3])
def test_engine_exact_panels_equal_row_major_exact(alg, overlap, monkeypatch):
    # a shard the engine keeps in panels in exact mode (>= 6144 rows, >= 2048 columns, a column
    # tail): y identical to the row-major exact kernels (MVG_NO_PANELS=1) and to the oracle,
    # across a redistribution with new values (the panel copy must be rebuilt), with the
    # distribution whole or in row chunks behind which the GEMVs run. The first multiply after
    # a distribution runs the row-major kernels, the second builds the panel copy and runs on
    # it: both ys are checked.
    R, Cn = 6160, 4098
    assert _lib.lib.mvg_exact_panel_width(R, Cn) > 0
    A1, x1 = signed(oracle.synth(R, Cn, 42), 1), signed(oracle.synth(1, Cn, 4242)[0], 2)
    A2, x2 = signed(oracle.synth(R, Cn, 43), 3), signed(oracle.synth(1, Cn, 4243)[0], 4)
    ys = {}
    for no_panels in ("0", "1"):
        monkeypatch.setenv("MVG_NO_PANELS", no_panels)
        c = mm.Comm.init_all([0])
        try:
            with mm.Multiplier(alg, R, Cn, c, exact=True) as e:
                e.set_overlap(overlap)
                out = []
                for A, x in ((A1, x1), (A2, x2)):
                    e.distribute(A, x)
                    e.multiply()
                    out.append(e.collect())
                    assert e.exact_panel_width() == 0 or A is A2  # allocated by the 2nd multiply
                    e.multiply()
                    out.append(e.collect())
                    assert (e.exact_panel_width() > 0) == (no_panels == "0")
                ys[no_panels] = out
        finally:
            c.destroy()
    for i, (A, x) in enumerate(((A1, x1), (A1, x1), (A2, x2), (A2, x2))):
        want = oracle.multiply_std_rowwise(A, x)
        assert np.array_equal(ys["1"][i], want), (alg, i)
        assert np.array_equal(ys["0"][i], want), (alg, i)


def test_engine_exact_panels_fill_synth_and_toggle(comm1):
    # device-resident inputs: exact on (row-major first, then panels built by the second
    # multiply), off (tree kernel on dA, panel copy released), on again (rebuilt at once: dA has
    # been multiplied since the fill) — sampled rows against the oracle bit for bit
    R, Cn = 8192, 4096
    with mm.Multiplier("rowwise", R, Cn, comm1) as e:
        e.fill_synth()
        e.set_exact(True)
        e.multiply()
        y0 = e.collect()
        assert e.exact_panel_width() == 0  # a fill multiplied once: no panel copy yet
        e.multiply()
        y1 = e.collect()
        assert e.exact_panel_width() == 256
        e.set_exact(False)
        assert e.exact_panel_width() == 0
        e.multiply()
        yt = e.collect()
        e.set_exact(True)
        e.multiply()
        y2 = e.collect()
    assert np.array_equal(y0, y1) and np.array_equal(y1, y2)
    assert max_rel(yt, y1) <= 1e-12
    x = oracle.synth(1, Cn, mm.SEED_X)[0]
    for r in [0, 1, 7, 8, R // 2, R - 1]:
        Ar = oracle.synth_block(r, 1, 0, Cn, Cn, mm.SEED_A)
        assert oracle.multiply_std_rowwise(Ar, x)[0] == y1[r], r


def _hip_runtime():
    """The HIP runtime libmatvec_gpu.so runs on, through ctypes. PyTorch's wheel ships its own
    libamdhip64 with the same soname (libamdhip64.so.7); the package loads PyTorch first, so the
    library's dependency resolves to that copy and the process maps one HIP runtime. Without
    PyTorch (MVG_NO_TORCH=1) it is the loader's resolution of the library's own dependency."""
    import ctypes
    import subprocess

    mapped = {os.path.realpath(ln.split()[-1]) for ln in open("/proc/self/maps") if "libamdhip64" in ln}
    if len(mapped) == 1:
        return ctypes.CDLL(mapped.pop())
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    path = next(ln.split("=>")[1].split("(")[0].strip() for ln in out.splitlines() if "libamdhip64" in ln)
    assert os.path.realpath(path) in mapped, (path, mapped)
    return ctypes.CDLL(path)


@pytest.fixture
def exact_hooks():
    lib = _lib.lib
    yield lib
    lib.mvg_debug_set_cu_count(0)
    lib.mvg_debug_set_exact_even_lds(0)


def test_exact_dispatch_falls_back_when_the_runtime_refuses_the_lds_reservation(exact_hooks):
    """The evenly placed form reserves LDS to place one 8-wave workgroup per CU. A runtime that
    turns the reservation down (forced here: 200 KiB, above the CU's 160 KiB) gets the one-wave
    form's sums — the reference's, bit for bit — and the dispatch keeps to the one-wave form on
    the device from then on (auto_variant says so; no failing launch per call)."""
    lib = exact_hooks
    _lib.check(lib.mvg_debug_set_cu_count(32), "cu count")  # 6144 rows = 96 workgroups = 3 rounds
    m, k = 6144, 1000
    name = lambda: lib.mvg_gemv_exact_variant_name(lib.mvg_gemv_exact_auto_variant(k, m, k)).decode()  # noqa: E731
    assert name() == "hop8e_l8_w2_u16_n8"
    A = signed(oracle.synth(m, k, 42), 5)
    x = signed(oracle.synth(1, k, 4242)[0], 6)
    want = oracle.multiply_std_rowwise(A, x)
    assert np.array_equal(mm.multiply_std_rowwise(A, x, exact=True), want)  # the even form itself
    _lib.check(lib.mvg_debug_set_exact_even_lds(200 * 1024), "even lds")
    assert name() == "hop8e_l8_w2_u16_n8"  # not refused yet
    y = mm.multiply_std_rowwise(A, x, exact=True)
    assert np.array_equal(y, want), max_rel(y, want)
    assert name() == "hop8_l8_w2_u16"  # the refusal is remembered for this device
    dev = ctypes.c_int(0)
    assert _hip_runtime().hipGetDevice(ctypes.byref(dev)) == 0
    assert lib.mvg_gemv_exact_even_refused(dev.value) == 1  # and visible to the caller (bench records it)
    assert np.array_equal(mm.multiply_std_rowwise(A, x, exact=True), want)
    _lib.check(lib.mvg_debug_set_exact_even_lds(0), "even lds")  # forgets the refusal
    assert name() == "hop8e_l8_w2_u16_n8" and lib.mvg_gemv_exact_even_refused(dev.value) == 0
    assert lib.mvg_gemv_exact_even_refused(64) == _lib.MVG_E_INVALID


def test_exact_call_reports_an_error_pending_from_an_earlier_call(exact_hooks):
    """An error an earlier HIP call left pending is returned by the next exact call as a
    failure (never taken for a refused launch and silently re-dispatched); the call after that
    runs normally."""
    lib = exact_hooks
    m, k = 6144, 1000
    A = oracle.synth(m, k, 42)
    x = oracle.synth(1, k, 4242)[0]
    dA, dx, dy = mm.DeviceBuffer(m * k).upload(A), mm.DeviceBuffer(k).upload(x), mm.DeviceBuffer(m)
    try:
        _lib.check(lib.mvg_stream_sync(None), "sync")
        hip = _hip_runtime()
        assert hip.hipSetDevice(1 << 20) != 0  # no such device: leaves an error pending
        rc = lib.mvg_gemv_exact(dA.ptr, k, dx.ptr, dy.ptr, m, k, None)
        assert rc != 0 and "pending" in lib.mvg_last_error().decode()
        _lib.check(lib.mvg_gemv_exact(dA.ptr, k, dx.ptr, dy.ptr, m, k, None), "mvg_gemv_exact")
        _lib.check(lib.mvg_stream_sync(None), "sync")
        assert np.array_equal(dy.download(m), oracle.multiply_std_rowwise(A, x))
    finally:
        for b in (dA, dx, dy):
            b.free()


def test_every_launch_entry_reports_an_error_pending_from_an_earlier_call():
    """The tree, multi-vector, exact, panel and relayout entry points all take an error an
    earlier HIP call left pending first and report it as that call's (nothing launched), so the
    same stale error is attributed the same way whichever kernel the engine calls next."""
    lib = _lib.lib
    m, k, P = 6144, 1024, 256
    A = oracle.synth(m, k, 42)
    x = oracle.synth(1, k, 4242)[0]
    dA, dx, dy = mm.DeviceBuffer(m * k).upload(A), mm.DeviceBuffer(k).upload(x), mm.DeviceBuffer(2 * m)
    dAp, dX = mm.DeviceBuffer(m * k), mm.DeviceBuffer(2 * k)
    dX.upload(np.concatenate([x, x]))
    calls = {
        "mvg_gemv": lambda: lib.mvg_gemv(dA.ptr, k, dx.ptr, dy.ptr, m, k, None),
        "mvg_gemv_multi": lambda: lib.mvg_gemv_multi(dA.ptr, k, dX.ptr, k, dy.ptr, m, m, k, 2, None),
        "mvg_gemv_exact": lambda: lib.mvg_gemv_exact(dA.ptr, k, dx.ptr, dy.ptr, m, k, None),
        "mvg_panel_relayout": lambda: lib.mvg_panel_relayout(dA.ptr, k, m, k, dAp.ptr, m * P, P, None),
        "mvg_gemv_exact_panels": lambda: lib.mvg_gemv_exact_panels(dAp.ptr, m * P, P, dx.ptr, dy.ptr, m, k, 0, None),
    }
    try:
        hip = _hip_runtime()
        for where, call in calls.items():
            _lib.check(lib.mvg_stream_sync(None), "sync")
            assert hip.hipSetDevice(1 << 20) != 0  # no such device: leaves an error pending
            rc = call()
            err = lib.mvg_last_error().decode()
            assert rc == _lib.MVG_E_HIP and err.startswith(where + ": HIP error pending"), (where, rc, err)
            _lib.check(call(), where)  # the next call runs normally
        _lib.check(lib.mvg_stream_sync(None), "sync")
        assert np.array_equal(dy.download(m), oracle.multiply_std_rowwise(A, x))  # the panels' exact y
    finally:
        for b in (dA, dx, dy, dAp, dX):
            b.free()
