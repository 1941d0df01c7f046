"""C-ABI library: loads, exports every declared symbol, and its host-only logic (planner,
exchange schedule, synthetic generator, text I/O) matches the reference's behaviour. No GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN_DIR, REPO
from matvec_mpi_multiplier_amd import _lib
from matvec_mpi_multiplier_amd import multiplier as mm
from oracle import oracle

HEADER = os.path.join(REPO, "include", "matvec_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mvg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 40
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes binding covers the whole header
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_built_for_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_errors():
    assert b"gfx950" in _lib.lib.mvg_version()
    assert _lib.lib.mvg_strerror(_lib.MVG_E_INDIVISIBLE) == b"shape does not divide over the rank count"
    rc = _lib.lib.mvg_plan_shard(0, 10, 10, 3, 0, C.byref(_lib.Shard()))
    assert rc == _lib.MVG_E_INDIVISIBLE
    assert b"10 mod 3 = 1. Unable to parallellize task." == _lib.lib.mvg_last_error()


@pytest.mark.parametrize("p", list(range(1, 130)))
def test_grid_shape_matches_reference(p):
    assert mm.get_2_most_closest_multipliers(p) == oracle.grid_shape(p)


def test_grid_shape_rejects_nonpositive():
    with pytest.raises(_lib.MvgError):
        mm.get_2_most_closest_multipliers(0)


# ---------------------------------------------------------------- shard planner
def _tiles(alg, R, Cn, P):
    return [mm.plan_shard(alg, R, Cn, P, r) for r in range(P)]


@pytest.mark.parametrize("R,Cn,P", [(4, 8, 2), (480, 480, 6), (120, 6000, 8), (960, 96, 3), (16384, 16384, 8),
                                    (4194304, 512, 8), (131072, 131072, 8), (65536, 65536, 8)])
def test_shards_tile_the_matrix(R, Cn, P):
    for alg in ("rowwise", "colwise", "blockwise"):
        try:
            shards = _tiles(alg, R, Cn, P)
        except _lib.IndivisibleError:
            continue
        cover = sum(s.n_rows * s.n_cols for s in shards)
        assert cover == R * Cn
        # disjoint: distinct (row_off, col_off) origins on a regular grid
        assert len({(s.row_off, s.col_off) for s in shards}) == P
        for s in shards:
            assert 0 <= s.row_off and s.row_off + s.n_rows <= R
            assert 0 <= s.col_off and s.col_off + s.n_cols <= Cn


def test_rowwise_plan_is_scatter_order():
    s = _tiles("rowwise", 12, 5, 3)
    assert [(t.row_off, t.n_rows, t.col_off, t.n_cols, t.y_off, t.y_len) for t in s] == [
        (0, 4, 0, 5, 0, 4), (4, 4, 0, 5, 4, 4), (8, 4, 0, 5, 8, 4)]


def test_colwise_plan_is_strip_order():
    s = _tiles("colwise", 3, 12, 4)
    assert [(t.col_off, t.n_cols, t.n_rows, t.y_len) for t in s] == [(0, 3, 3, 3), (3, 3, 3, 3), (6, 3, 3, 3), (9, 3, 3, 3)]


def test_blockwise_plan_is_rank_i_times_c_plus_j():
    # multiplier_blockwise.c:56,71: block (i, j) goes to rank i*c + j on the r x c grid
    s = _tiles("blockwise", 8, 12, 8)  # 2 x 4 grid
    for t in s:
        assert (t.grid_rows, t.grid_cols) == (2, 4)
        assert t.rank == t.grid_r * 4 + t.grid_c
        assert (t.row_off, t.col_off, t.n_rows, t.n_cols) == (t.grid_r * 4, t.grid_c * 3, 4, 3)


def test_divisibility_errors_match_reference_checks():
    # rowwise.c:72 R % P; colwise.c:151 C % P; blockwise.c:278 (R*C) % P
    with pytest.raises(_lib.IndivisibleError):
        mm.plan_shard("rowwise", 10, 8, 4, 0)
    mm.plan_shard("rowwise", 12, 7, 4, 0)
    with pytest.raises(_lib.IndivisibleError):
        mm.plan_shard("colwise", 8, 10, 4, 0)
    mm.plan_shard("colwise", 7, 12, 4, 0)
    with pytest.raises(_lib.IndivisibleError):
        mm.plan_shard("blockwise", 5, 5, 2, 0)


def test_blockwise_refuses_ragged_grid_the_reference_truncates():
    # 3 x 8 at P=4 passes the reference's (R*C) % P check but R % 2 != 0: the reference drops
    # a row (SURVEY §4 bug 1); the planner refuses (deliberate deviation).
    with pytest.raises(_lib.IndivisibleError):
        mm.plan_shard("blockwise", 3, 8, 4, 0)
    with pytest.raises(_lib.IndivisibleError):
        mm.plan_shard("blockwise", 4, 5, 4, 0)


def test_plan_rejects_bad_arguments():
    for args in [(0, 4, 4, 0, 0), (0, 4, 4, 2, 2), (0, -1, 4, 1, 0), (9, 4, 4, 1, 0)]:
        with pytest.raises(_lib.MvgError):
            mm.plan_shard(*args)


def test_empty_shapes_plan():
    s = mm.plan_shard("rowwise", 0, 5, 2, 1)
    assert s.n_rows == 0
    assert mm.plan_shard("colwise", 3, 0, 1, 0).n_cols == 0


# ---------------------------------------------------------------- exchange schedule
def test_exchange_rowwise_and_colwise():
    for r in range(4):
        (st,) = mm.plan_exchange("rowwise", 16, 8, 4, r)
        assert (st.op, st.comm, st.member, st.root, st.count, st.src, st.dst) == (
            _lib.X_GATHER, _lib.X_WORLD, 1, 0, 4, _lib.X_BUF_PART, _lib.X_BUF_Y)
        (st,) = mm.plan_exchange("colwise", 16, 8, 4, r)
        assert (st.op, st.comm, st.count) == (_lib.X_REDUCE, _lib.X_WORLD, 16)


def test_exchange_blockwise_two_level():
    for r in range(8):  # 2 x 4 grid
        red, gat = mm.plan_exchange("blockwise", 16, 16, 8, r)
        gi, gj = divmod(r, 4)
        assert (red.op, red.comm, red.color, red.key, red.member, red.count) == (_lib.X_REDUCE, _lib.X_ROW, gi, gj, 1, 8)
        assert red.dst == _lib.X_BUF_ROW
        assert (gat.op, gat.comm, gat.key, gat.member, gat.src, gat.dst) == (
            _lib.X_GATHER, _lib.X_COL, gi, int(gj == 0), _lib.X_BUF_ROW, _lib.X_BUF_Y)


def test_exchange_blockwise_single_grid_row_reduces_into_y():
    for r in range(3):  # 1 x 3 grid
        (red,) = mm.plan_exchange("blockwise", 6, 9, 3, r)
        assert red.comm == _lib.X_ROW and red.dst == _lib.X_BUF_Y


def test_exchange_solo_has_no_steps_unless_forced():
    for alg in ("rowwise", "colwise", "blockwise"):
        assert mm.plan_exchange(alg, 8, 8, 1, 0) == []
        assert len(mm.plan_exchange(alg, 8, 8, 1, 0, force_collect=True)) == 1


# ---------------------------------------------------------------- synthetic generator
def test_synth_host_matches_oracle_bit_exact():
    A = mm.synth_host(37, 129, 42)
    np.testing.assert_array_equal(A, oracle.synth(37, 129, 42))
    blk = oracle.synth_block(5, 7, 100, 29, 129, 42)
    np.testing.assert_array_equal(A[5:12, 100:129], blk)
    assert _lib.lib.mvg_synth_value(4242, 17) == oracle.synth_value(4242, 17)


def test_synth_large_index_matches_oracle():
    for idx in (0, 1, 2**32 - 1, 2**32 + 7, 131072 * 131072 - 1, 2**62 + 3):
        assert _lib.lib.mvg_synth_value(42, idx) == oracle.synth_value(42, idx)


# ---------------------------------------------------------------- text I/O
def test_filenames_match_reference():
    assert mm.build_matrix_filename(4, 8) == "matrix_4_8.txt"
    assert mm.build_vector_filename(8) == "vector_8.txt"
    assert mm.build_matrix_filename(131072, 131072) == "matrix_131072_131072.txt"


def test_load_reference_fixture():
    A = mm.load_matr(4, 8, GOLDEN_DIR)
    x = mm.load_vec(8, GOLDEN_DIR)
    np.testing.assert_array_equal(A, np.loadtxt(os.path.join(GOLDEN_DIR, "matrix_4_8.txt")))
    np.testing.assert_array_equal(x, np.arange(1, 9, dtype=np.float64))


def test_missing_file_is_io_error(tmp_path):
    with pytest.raises(_lib.MvgError) as e:
        mm.load_matr(3, 3, str(tmp_path))
    assert e.value.code == _lib.MVG_E_IO


def test_short_file_is_io_error(tmp_path):
    (tmp_path / "vector_5.txt").write_text("1.0 2.0 3.0\n")
    with pytest.raises(_lib.MvgError) as e:
        mm.load_vec(5, str(tmp_path))
    assert e.value.code == _lib.MVG_E_IO


def test_non_numeric_token_is_io_error(tmp_path):
    (tmp_path / "vector_3.txt").write_text("1.0 abc 3.0\n")
    with pytest.raises(_lib.MvgError):
        mm.load_vec(3, str(tmp_path))


def test_free_form_whitespace_and_extra_tokens(tmp_path):
    # fscanf("%lf") reads whitespace-separated tokens regardless of line layout and stops
    # after R*C values (matr_utils.c:55-59)
    (tmp_path / "matrix_2_3.txt").write_text("  1.5\t2.25\n\n3e-1 4\r\n5.0000 -6.125 99 100\n")
    A = mm.load_matr(2, 3, str(tmp_path))
    np.testing.assert_array_equal(A, [[1.5, 2.25, 0.3], [4.0, 5.0, -6.125]])


def test_synth_text_roundtrip_parallel_parser(tmp_path):
    # > 1 MiB so the parser splits the file over threads; bit-exact vs the generator
    R, Cn = 300, 700
    mm.write_matr_synth(str(tmp_path / f"matrix_{R}_{Cn}.txt"), R, Cn, 42)
    A = mm.load_matr(R, Cn, str(tmp_path))
    np.testing.assert_array_equal(A, oracle.synth(R, Cn, 42))
    np.testing.assert_array_equal(A, np.loadtxt(tmp_path / f"matrix_{R}_{Cn}.txt"))


def test_parser_is_bit_identical_to_strtod(tmp_path):
    # the loader's exact fast path (Clinger: short decimal tokens) and its strtod fallback must
    # give the double strtod/fscanf("%lf") gives for every token; Python's float() is correctly
    # rounded, as glibc's strtod is
    rng = np.random.default_rng(7)
    vals = np.concatenate([rng.uniform(-1e6, 1e6, 3000), rng.uniform(0, 1, 3000),
                           rng.standard_normal(2000) * 10.0 ** rng.integers(-30, 30, 2000)])
    toks = [f"{v:.4f}" for v in vals[:6000]]                      # the reference's format
    toks += [f"{v:.17g}" for v in vals] + [f"{v:.18e}" for v in vals[::3]] + [f"{v:.6g}" for v in vals[::2]]
    toks += [str(int(v)) for v in vals[:500]] + [f"{v:.2f}E+3" for v in vals[:300]]
    toks += ["0", "-0", "-0.0", "+5", ".5", "5.", "-.25", "1e22", "1e23", "1e-22", "1e-23", "22e-22",
             "9007199254740992", "9007199254740993", "9007199254740993e-5", "0.000000000000000000000001",
             "123456789012345678901234567890", "1234567890123456789", "12345678901234567890e-30",
             "1E5", "4.9e-324", "1.7976931348623157e308", "2.2250738585072014e-308", "1e400", "-1e-400",
             "0.10000000000000000555", "100000000000000000000000", "3.0000000000000000000000001",
             "inf", "-inf", "Infinity", "0x1.8p1", "00000000000000000000000012.5000000000000000000000"]
    (tmp_path / f"vector_{len(toks)}.txt").write_text("\n".join(toks) + "\n")
    got = mm.load_vec(len(toks), str(tmp_path))
    want = np.array([float.fromhex(t) if t.startswith("0x") else float(t) for t in toks])
    bad = [t for t, g, w in zip(toks, got.view(np.uint64), want.view(np.uint64)) if g != w]
    assert not bad, bad[:10]


def test_parser_plain_tokens_many_ranges(tmp_path):
    # the 8-bytes-at-a-time path for [-]digits[.digits] tokens: every fraction length 0 ... 9
    # (8 and more leave it for the general path), 1 ... 16 digits in all (15 is its limit),
    # mixed separators, over a multi-MiB file so that every thread's four interleaved ranges and
    # their cut points are exercised; the last token ends the file without a newline, fewer
    # than 8 bytes after its point
    rng = np.random.default_rng(11)
    toks = []
    for i in range(400_000):
        ni, nf = int(rng.integers(0, 10)), int(rng.integers(0, 10))
        ip = "".join(str(d) for d in rng.integers(0, 10, ni))
        fp = "".join(str(d) for d in rng.integers(0, 10, nf))
        t = (ip or ("0" if nf == 0 else "")) + ("." + fp if nf or i % 7 == 0 else "")
        toks.append(("-" if i % 3 == 0 else "") + t)
    toks += ["123456789012345", "12345678901234.5", "1234567890123456", "0.000000000000001", "-0.0000",
             "7.", ".5", "-.5"]
    seps = [" ", "\n", "\t", "\r\n", "  "]
    text = "".join(t + seps[i % len(seps)] for i, t in enumerate(toks)) + "3.25"
    toks.append("3.25")
    (tmp_path / f"vector_{len(toks)}.txt").write_text(text)
    got = mm.load_vec(len(toks), str(tmp_path))
    want = np.array([float(t) for t in toks])
    bad = [t for t, g, w in zip(toks, got.view(np.uint64), want.view(np.uint64)) if g != w]
    assert not bad, bad[:10]


def test_write_vec_roundtrips(tmp_path):
    v = np.array([222.19999999999999, 1e-300, -0.0, 3.141592653589793, 1076.4842229100022])
    mm.write_vec(str(tmp_path / "vector_5.txt"), v)
    np.testing.assert_array_equal(mm.load_vec(5, str(tmp_path)), v)


def test_binary_cache_written_used_and_invalidated(tmp_path, monkeypatch):
    R, Cn = 40, 30
    txt = tmp_path / f"matrix_{R}_{Cn}.txt"
    binp = tmp_path / f"matrix_{R}_{Cn}.bin"
    mm.write_matr_synth(str(txt), R, Cn, 42)
    want = oracle.synth(R, Cn, 42)
    monkeypatch.setenv("MVG_BIN_CACHE", "1")
    np.testing.assert_array_equal(mm.load_matr(R, Cn, str(tmp_path)), want)
    assert binp.exists() and binp.stat().st_size == 24 + R * Cn * 8
    # the cache is what gets read while it is not older than the text
    monkeypatch.delenv("MVG_BIN_CACHE")
    txt.write_text("1.0 " * (R * Cn))
    os.utime(txt, (binp.stat().st_mtime - 10, binp.stat().st_mtime - 10))
    np.testing.assert_array_equal(mm.load_matr(R, Cn, str(tmp_path)), want)
    # a newer text invalidates it; MVG_BIN_CACHE=0 ignores it
    os.utime(txt, (binp.stat().st_mtime + 10, binp.stat().st_mtime + 10))
    np.testing.assert_array_equal(mm.load_matr(R, Cn, str(tmp_path)), np.ones((R, Cn)))
    os.utime(txt, (binp.stat().st_mtime - 10, binp.stat().st_mtime - 10))
    monkeypatch.setenv("MVG_BIN_CACHE", "0")
    np.testing.assert_array_equal(mm.load_matr(R, Cn, str(tmp_path)), np.ones((R, Cn)))


def test_binary_cache_shape_mismatch_falls_back_to_text(tmp_path):
    mm.write_matr_synth(str(tmp_path / "matrix_4_6.txt"), 4, 6, 42)
    mm.write_matr_bin(str(tmp_path / "matrix_4_6.bin"), np.zeros((6, 4)))  # wrong shape in header
    np.testing.assert_array_equal(mm.load_matr(4, 6, str(tmp_path)), oracle.synth(4, 6, 42))


def test_speedup_efficiency_tables(tmp_path):
    from matvec_mpi_multiplier_amd import stats

    # the executables' header (with spaces) and the reference's published one (without)
    (tmp_path / "a.csv").write_text("n_rows, n_cols, n_processes, time\n600, 600, 1, 0.002\n600, 600, 2, 0.001\n"
                                    "600, 600, 4, 0.0008\n")
    (tmp_path / "b.csv").write_text("n_rows,n_cols,n_processes,time\n600,600,1,0.002\n600,600,2,0.001\n")
    for f in ("a.csv", "b.csv"):
        t = stats.read_times(str(tmp_path / f))
        rows = stats.speedup_efficiency(t[(600, 600)])
        assert rows[0] == {"p": 1, "time": 0.002, "speedup": 1.0, "efficiency": 1.0}
        assert rows[1]["speedup"] == pytest.approx(2.0) and rows[1]["efficiency"] == pytest.approx(1.0)
    assert "| 600 | 600 | 4 | 0.000800 | 2.500 | 0.625 |" in stats.table(str(tmp_path / "a.csv"))


def test_host_first_touch_zeroes_the_range_without_numa_info():
    """mvg_host_first_touch (NUMA placement of the executables' shared window) zeroes exactly
    the given range, in parallel above 64 MiB, and still does so when the GPU's NUMA node cannot
    be found (no GPU here: the caller's CPUs touch the pages)."""
    a = np.full(20_000_000, 7.0)  # 160 MB: the threaded path
    off, n = 1000, 19_000_000
    assert _lib.lib.mvg_host_first_touch(a[off:].ctypes.data, n * 8, 0) == 0
    assert not a[off:off + n].any()
    assert (a[:off] == 7.0).all() and (a[off + n:] == 7.0).all()
    small = np.full(1000, 3.0)
    assert _lib.lib.mvg_host_first_touch(small.ctypes.data, small.nbytes, 0) == 0 and not small.any()


# dispatch is host logic (no GPU needed): the names the auto choice resolves to per shape
def test_auto_variant_names_match_the_dispatch_table():
    names = {k: _lib.lib.mvg_gemv_variant_name(_lib.lib.mvg_gemv_auto_variant(k, m, k)).decode()
             for m, k in ((16384, 16384), (65536, 32768), (65536, 8192), (524288, 4096), (2097152, 1024),
                          (4194304, 512))}
    assert names[16384] == "rowblk_w4_r2_u8" and names[32768] == "rowblk_w4_r2_u8"
    assert names[8192] == "rowblk_w8_r2_u4" and names[512] == "vec_l64_r1_u4_nt1_o5"
    pick = lambda m, k: _lib.lib.mvg_gemv_variant_name(_lib.lib.mvg_gemv_auto_variant(k, m, k)).decode()
    assert pick(120, 60000) == "rowblk_w4_r2_u4_splitk" and pick(1024, 131072) == "rowblk_w4_r2_u4_splitk"
    assert pick(4096, 16384) == "rowblk_w4_r2_u8" and pick(1536, 32768) == "rowblk_w4_r2_u8"
    # below 1 GiB with 768 < K < 8192: row-per-workgroup forms (the reference's test.sh squares)
    assert pick(4200, 4200) == "rowblk_w2_r2_u4" and pick(1800, 1800) == "rowblk_w2_r2_u4"
    assert pick(1024, 6144) == "rowblk_w2_r2_u4"
    # rows off the 128-B lines (lda not a multiple of 16), long and many: line-aligned row pairs
    assert pick(7800, 7800) == "rowlines_w8_u4_x0" and pick(10200, 10200) == "rowlines_w8_u4_x0"
    assert pick(16384, 16386) == "rowlines_w8_u4_x0" and pick(16384, 16400) == "rowblk_w4_r2_u8"
    assert names[4096] == "rowblk_w8_r2_u4" and names[1024] == "vec_l64_r4_u4_nt1_o5"
    # aligned rows keep the plain workgroup order (the XCD-contiguous one gained < 2 %)
    assert pick(65536, 65536) == "rowblk_w4_r2_u8" and pick(131072, 131072) == "rowblk_w4_r2_u8"
    assert pick(131072, 32768) == "rowblk_w4_r2_u8" and pick(131072, 16384) == "rowblk_w4_r2_u8"
    assert pick(65536, 16384) == "rowblk_w4_r2_u8"
    assert pick(32768, 8192) == "rowblk_w8_r2_u4" and pick(16384, 8192) == "rowblk_w8_r2_u4"
    # A >= 1 GiB, 4096 <= K < 8192: the row-block form; K <= 3072 keeps the wave-owns-rows form
    assert pick(131072, 3072) == "vec_l64_r2_u4_nt1_o7" and pick(1048576, 2048) == "vec_l64_r2_u4_nt1_o7"
    assert pick(65536, 4200) == "rowblk_w8_r2_u4" and pick(8388608, 4096) == "rowblk_w8_r2_u4"
    assert pick(8388608, 3072) == "vec_l64_r2_u4_nt1_o7"
    # odd widths (odd lda): the 16-B kernels through unaligned loads, not the 8-B ones
    assert pick(16384, 16383) == "rowlines_w8_u4_x0" and pick(65536, 8191) == "rowlines_w8_u4_x0"
    assert pick(2048, 65535) == "rowblk_w4_r2_u8_xcd"
    assert pick(1200, 60001) == "rowblk_w4_r2_u4_splitk" and pick(10200, 1275) == "rowblk_w2_r2_u4"
    assert pick(4200, 525) == "vec_l64_r4_u4_nt1_o0" and pick(524288, 511) == "vec_l64_r4_u4_nt1_o0"


def test_exact_panel_dispatch_and_argument_checks():
    # host-only parts of the column-panel exact path: where the engine keeps a
    # panel copy, which variant runs it, and the argument checks that refuse before any launch
    lib = _lib.lib
    width = lib.mvg_exact_panel_width
    assert width(16384, 16384) == 256            # config 2
    assert width(65536, 32768) == 256            # config 4's block at G = 8 (16 GiB)
    assert width(65536, 8192) == 256             # config 3's strip at G = 8
    assert width(10200, 10200) == 256 and width(7800, 7800) == 256  # the reference's sizes
    assert width(65536, 65536) == 0              # above 16 GiB: row-major forms
    assert width(131072, 131072) == 0
    assert width(8192, 16384) == 0               # few rows, long rows
    assert width(6144, 2048) == 0                # under 128 MiB
    assert width(4096, 65536) == 0 and width(4194304, 512) == 0  # few rows / short rows
    name = lambda m, k: lib.mvg_gemv_exact_panel_variant_name(lib.mvg_gemv_exact_panel_auto_variant(m, k)).decode()  # noqa: E731
    assert name(16384, 16384) == "panel_l8_w2_u8" and name(65536, 8192) == "panel_l8_w2_u8"
    names = [lib.mvg_gemv_exact_panel_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_panel_variant_count())]
    assert names[0] == "auto" and all(n.startswith("panel_l") for n in names[1:])
    assert lib.mvg_gemv_exact_panel_variant_name(len(names)) == b"invalid"
    fake = 1 << 20  # never dereferenced: every call below is refused before a launch
    bad = [
        lib.mvg_gemv_exact_panels(fake, 256 * 64, 96, fake, fake, 64, 1000, 0, None),       # P not a power of 2
        lib.mvg_gemv_exact_panels(fake, 256 * 64, 8, fake, fake, 64, 1000, 0, None),        # P < segment
        lib.mvg_gemv_exact_panels(fake, 256 * 64 - 1, 256, fake, fake, 64, 1000, 0, None),  # pstride < m*P
        lib.mvg_gemv_exact_panels(fake + 8, 256 * 64, 256, fake, fake, 64, 1000, 0, None),  # A off 16 B
        lib.mvg_gemv_exact_panels(fake, 256 * 64, 256, fake + 8, fake, 64, 1000, 0, None),  # x off 16 B
        lib.mvg_gemv_exact_panels(fake, 256 * 64, 256, fake, fake, -1, 1000, 0, None),      # negative m
        lib.mvg_gemv_exact_panels(fake, 256 * 64, 256, fake, fake, 64, 1000, len(names), None),  # variant
        lib.mvg_gemv_exact_panels(None, 256 * 64, 256, None, fake, 64, 1000, 0, None),      # null A, x
        lib.mvg_panel_relayout(fake, 999, 64, 1000, fake, 256 * 64, 256, None),             # lda < k
        lib.mvg_panel_relayout(fake, 1000, 64, 1000, fake, 256 * 64, 100, None),            # P not 2^n
        lib.mvg_panel_relayout(fake, 1000, 64, 1000, fake, 256 * 63, 256, None),            # pstride
        lib.mvg_panel_relayout(None, 1000, 64, 1000, fake, 256 * 64, 256, None),            # null
    ]
    assert all(rc == _lib.MVG_E_INVALID for rc in bad), bad
    # nothing to do is not an error (no launch either)
    assert lib.mvg_gemv_exact_panels(None, 0, 256, None, None, 0, 1000, 0, None) == 0
    assert lib.mvg_panel_relayout(None, 0, 0, 0, None, 0, 256, None) == 0


def test_gendata_writes_the_reference_inputs(tmp_path):
    # python -m matvec_mpi_multiplier_amd.gendata: ./data/matrix_R_C.txt + vector_C.txt in the
    # reference's "%.4f" format (the generator its repository lacks), values = the synthetic spec
    from matvec_mpi_multiplier_amd import gendata
    from oracle import oracle

    d = str(tmp_path / "data")
    gendata.main(["6", "10", "3", "10", "--dir", d])
    assert sorted(os.listdir(d)) == ["matrix_3_10.txt", "matrix_6_10.txt", "out", "vector_10.txt"]
    np.testing.assert_array_equal(mm.load_matr(6, 10, d), oracle.synth(6, 10, 42))
    np.testing.assert_array_equal(mm.load_matr(3, 10, d), oracle.synth(3, 10, 42))
    np.testing.assert_array_equal(mm.load_vec(10, d), oracle.synth(1, 10, 4242)[0])
    assert open(os.path.join(d, "matrix_3_10.txt")).read().split()[0] == "%.4f" % oracle.synth(1, 1, 42)[0, 0]
    assert gendata.TEST_SH_SIZES == (600, 1800, 3000, 4200, 5400, 6600, 7800, 9000, 10200)
    with pytest.raises(SystemExit):
        gendata.main(["6"])


def test_multi_vector_dispatch_takes_dma_forms_on_long_rows():
    # gemv.hip pick_multi_dma: A through LDS by DMA (staggered starts) for vector groups on
    # long rows; the register forms elsewhere; never the DMA forms when 32 rows of lda exceed
    # the kernel's 32-bit offsets
    lib = _lib.lib
    name = lambda m, k, nv, lda=None: lib.mvg_gemv_multi_variant_name(
        lib.mvg_gemv_multi_auto_variant(lda or k, k, m, k, nv)).decode()
    assert name(16384, 16384, 8) == name(16384, 16384, 2) == name(2097152, 1024, 8) == "mdma_r2_t16_b2_w4_s5"
    assert name(4096, 65536, 4) == "mdma_r1_t16_b2_w4_s5"
    assert not name(4200, 4200, 8).startswith("mdma")
    assert not name(16384, 4096, 2).startswith("mdma")       # pairs: from K = 6144
    assert not name(4194304, 512, 8).startswith("mdma")      # short rows: x resident in LDS
    assert not name(16384, 16384, 8, lda=1 << 24).startswith("mdma")
    assert lib.mvg_gemv_multi_auto_variant(16384, 16384, 16384, 16384, 1) == 0
    # 9..16 vectors: one pass on the matrix cores where the DMA forms run
    assert name(16384, 16384, 16) == name(8192, 1024, 9) == "m16_r2_t16_b2_w4_s5"
    assert not name(4200, 4200, 16).startswith("m16")


@pytest.fixture
def cu_count():
    """The exact dispatch's CU count set through its test hook (mvg_debug_set_cu_count), put back
    to the device's afterwards."""
    yield lambda n: _lib.check(_lib.lib.mvg_debug_set_cu_count(n), "mvg_debug_set_cu_count")
    _lib.lib.mvg_debug_set_cu_count(0)


def test_exact_row_major_dispatch(cu_count):
    """pick_seq_variant (host logic) at the MI355X's 256 CUs, set explicitly (the device's own
    count on a GPU box, which a partitioned mode would change): the LDS form for line-aligned tall
    rows, the evenly placed 8-lane form where whole rounds of one 8-wave workgroup per CU cover
    the rows (16384·k rows, 768 < K < 65536), the one-wave 8-lane forms otherwise (partial rounds,
    short rows, K >= 65536), wider lane groups for few rows."""
    cu_count(256)
    name = lambda m, k, lda=None: _lib.lib.mvg_gemv_exact_variant_name(  # noqa: E731
        _lib.lib.mvg_gemv_exact_auto_variant(lda or k, m, k)).decode()
    assert name(16384, 16384) == "hop8e_l8_w2_u16_n8"     # config 2 (and its weak-scaled shards)
    assert name(16384, 16383) == "hop8e_l8_w2_u16_n8"     # odd width, same rows
    assert name(32768, 16384, 16386) == "hop8e_l8_w2_u16_n8"  # rows off the lines: no LDS form
    assert name(32768, 16384) == "seqx_r64_t16_b2_g8"     # line-aligned tall rows: the LDS form
    assert name(24576, 16384) == "hop8_l8_w2_u16"         # 1.5 rounds: a partial round costs a whole one
    assert name(65536, 65536) == "hop8_l8_w2_u24"         # K >= 65536
    assert name(131072, 131072) == "hop8_l8_w2_u24"
    assert name(524288, 512) == "hop8_l8_w2_u16"          # short rows want more waves per CU
    assert name(4194304, 512) == "hop8_l8_w2_u16"
    assert name(1200, 60000).startswith("hop8_l32")       # few long rows: the chain dominates


@pytest.mark.parametrize("cus", [256, 32, 100])
def test_exact_even_form_needs_whole_rounds_of_workgroups(cu_count, cus):
    """The evenly placed form's rule on its own: 64-row workgroups, one per CU per round, so it
    is taken exactly when the workgroup count is a positive multiple of the CU count (and
    768 < K < 65536, >= 6144 rows, no LDS form)."""
    cu_count(cus)
    for m in (6144, 8192, 16384, 24576, 32768 + 64, 49152):
        v = _lib.lib.mvg_gemv_exact_variant_name(_lib.lib.mvg_gemv_exact_auto_variant(16383, m, 16383)).decode()
        wgs = -(-m // 64)
        assert (v == "hop8e_l8_w2_u16_n8") == (wgs >= cus and wgs % cus == 0), (m, cus, v)



def test_runtime_info_names_the_bound_rccl_and_hip():
    """mvg_runtime_versions / mvg_runtime_path: the RCCL and HIP runtime this process's library
    calls go to (no device needed). Imported after PyTorch (the package's default), both are
    PyTorch's bundled copies, which satisfy the library's sonames."""
    info = _lib.runtime_info(hip_version=False)
    assert info["rccl_version_code"] and info["rccl_version"].count(".") == 2
    assert os.path.exists(info["rccl_path"]) and os.path.exists(info["hip_path"])
    assert os.path.basename(info["rccl_path"]).startswith("librccl.so")
    assert os.path.basename(info["hip_path"]).startswith("libamdhip64.so")
    # the bound copy is a mapped one, and only one copy of each is mapped
    real = lambda p: os.path.realpath(p)  # noqa: E731
    assert real(info["rccl_path"]) in {real(p) for p in info["mapped"]["librccl"]}
    assert len(info["mapped"]["libamdhip64"]) == 1 and len(info["mapped"]["librccl"]) == 1
    assert _lib.lib.mvg_runtime_path(7) == b""


def test_mapped_runtimes_and_version_text():
    maps = ["7f00-7f10 r-xp 00000000 08:01 123 /opt/rocm-7.2.0/lib/librccl.so.1.0.70200\n",
            "7f10-7f20 r--p 00000000 08:01 124 /usr/lib/python3/torch/lib/librccl.so\n",
            "7f20-7f30 r-xp 00000000 08:01 125 /usr/lib/python3/torch/lib/libamdhip64.so\n",
            "7f30-7f40 rw-p 00000000 00:00 0 \n", "7f40-7f50 r-xp 00000000 08:01 126 /usr/lib/librccl-net.so\n"]
    m = _lib.mapped_runtimes(maps)
    assert m["librccl"] == ["/opt/rocm-7.2.0/lib/librccl.so.1.0.70200", "/usr/lib/python3/torch/lib/librccl.so"]
    assert m["libamdhip64"] == ["/usr/lib/python3/torch/lib/libamdhip64.so"]
    assert _lib.rccl_version_text(22707) == "2.27.7" and _lib.rccl_version_text(22606) == "2.26.6"
