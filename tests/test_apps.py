"""The drop-in executables bin/multiplier_{rowwise,colwise,blockwise}: the reference's process
contract (argv, ./data inputs, messages, exit codes, ./data/out/<alg>.csv, y)."""
import os
import re
import shutil
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN_DIR, REPO, max_rel

ALGS = ("rowwise", "colwise", "blockwise")


def run(alg, args, cwd, **env):
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    return subprocess.run([os.path.join(REPO, "bin", f"multiplier_{alg}")] + [str(a) for a in args],
                          cwd=cwd, env=e, capture_output=True, text=True, timeout=300)


@pytest.fixture
def workdir(tmp_path):
    (tmp_path / "data" / "out").mkdir(parents=True)
    for f in ("matrix_4_8.txt", "vector_8.txt"):
        shutil.copy(os.path.join(GOLDEN_DIR, f), tmp_path / "data" / f)
    return tmp_path


def test_usage_without_arguments(workdir):
    r = run("rowwise", [], workdir)
    assert r.returncode == 1 and "usage" in r.stderr


@pytest.mark.parametrize("alg,R,C,G,msg", [
    ("rowwise", 4, 8, 3, "4 mod 3 = 1. Unable to parallellize task."),        # rowwise.c:72-75
    ("colwise", 4, 8, 3, "8 mod 3 = 2. Unable to parallellize task."),        # colwise.c:151-154
    ("blockwise", 5, 5, 2, "25 mod 2 = 1. Unable to parallellize task."),     # blockwise.c:277-281
    ("blockwise", 3, 8, 4, "3 x 8 does not split over a 2 x 2 grid."),       # deliberate deviation
])
def test_indivisible_prints_error_and_exits_zero(workdir, alg, R, C, G, msg):
    r = run(alg, [R, C], workdir, MVG_NGPUS=G)
    assert r.returncode == 0
    assert r.stdout.startswith("\nERROR!!!\n") and msg in r.stdout
    assert not (workdir / "data" / "out" / f"{alg}.csv").exists()  # the check precedes the CSV


def test_missing_input_file_message(workdir):
    r = run("rowwise", [6, 6], workdir, MVG_NGPUS=1)
    assert r.returncode == 0
    assert "Reading matrix from file './data/matrix_6_6.txt'..." in r.stdout
    assert "Unable to locate matrix file 'matrix_6_6.txt'" in r.stdout
    # the CSV header is created before the load, as in rowwise.c:77-88
    assert (workdir / "data" / "out" / "rowwise.csv").read_text() == "n_rows, n_cols, n_processes, time\n"


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ALGS)
def test_fixture_run_matches_reference(workdir, golden, alg):
    yout = workdir / "y.txt"
    r = run(alg, [4, 8], workdir, MVG_NGPUS=1, MVG_ITERS=5, MVG_Y_OUT=yout)
    assert r.returncode == 0, r.stderr
    assert "n_rows = 4\nn_cols = 8\n" in r.stdout
    assert "Reading vector from file './data/vector_8.txt'..." in r.stdout
    y = np.loadtxt(yout)
    assert max_rel(y, golden[f"fixture_4x8/{alg}/P1"]) <= 1e-12
    lines = (workdir / "data" / "out" / f"{alg}.csv").read_text().splitlines()
    assert lines[0] == "n_rows, n_cols, n_processes, time"
    assert re.fullmatch(r"4, 8, 1, \d+\.\d{6}", lines[1]), lines[1]
    # a second run appends a row (rowwise.c:163 opens with "a")
    run(alg, [4, 8], workdir, MVG_NGPUS=1, MVG_ITERS=2)
    assert len((workdir / "data" / "out" / f"{alg}.csv").read_text().splitlines()) == 3


@pytest.mark.gpu
def test_synthetic_large_run(workdir):
    from oracle import oracle

    R, C = 2048, 4096
    yout = workdir / "y.txt"
    r = run("colwise", [R, C], workdir, MVG_NGPUS=1, MVG_ITERS=3, MVG_SYNTH=1, MVG_Y_OUT=yout)
    assert r.returncode == 0, r.stderr
    assert "device-resident" in r.stdout
    y = np.loadtxt(yout)
    assert max_rel(y, oracle.multiply("colwise", oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0], 1)) <= 1e-12


def test_c_binding_example_is_plain_c():
    # examples/rowwise_binding.c builds with gcc -std=c99 against the header
    assert os.path.exists(os.path.join(REPO, "bin", "rowwise_binding"))


@pytest.mark.gpu
def test_c_binding_example_runs_the_fixture(workdir, golden):
    r = subprocess.run([os.path.join(REPO, "bin", "rowwise_binding"), "4", "8", "1"], cwd=workdir,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    y = np.array([float(v) for v in r.stdout.split()[-4:]])
    assert max_rel(y, golden["fixture_4x8/rowwise/P1"]) <= 1e-12
    assert re.fullmatch(r"4, 8, 1, \d+\.\d{6}\n", r.stderr.splitlines()[-1] + "\n")
    # the same C program with MVG_EXACT=1: the reference's digits exactly
    r = subprocess.run([os.path.join(REPO, "bin", "rowwise_binding"), "4", "8", "1"], cwd=workdir,
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, MVG_EXACT="1"))
    assert r.returncode == 0, r.stderr
    assert r.stdout.split()[-4:] == ["%.17g" % v for v in golden["fixture_4x8/rowwise/P1"]]


# ---- launched like the reference: mpiexec -n P bin/multiplier_<alg> R C (test.sh:11)
MPIEXEC = "/opt/conda/bin/mpiexec"
needs_mpiexec = pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no MPI launcher in this image")


def mpirun(alg, np_, args, cwd, **env):
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    return subprocess.run([MPIEXEC, "-n", str(np_), os.path.join(REPO, "bin", f"multiplier_{alg}")]
                          + [str(a) for a in args], cwd=cwd, env=e, capture_output=True, text=True, timeout=300)


@needs_mpiexec
@pytest.mark.parametrize("alg,R,C,P,msg", [
    ("rowwise", 4, 8, 3, "4 mod 3 = 1. Unable to parallellize task."),
    ("colwise", 4, 8, 3, "8 mod 3 = 2. Unable to parallellize task."),
    ("blockwise", 5, 5, 2, "25 mod 2 = 1. Unable to parallellize task."),
])
def test_mpiexec_indivisible_root_prints_every_rank_exits_zero(workdir, alg, R, C, P, msg):
    # P comes from the launcher, as in the reference; only the root prints, and unlike the
    # reference (whose other ranks are left waiting in MPI_Barrier) every rank exits 0
    r = mpirun(alg, P, [R, C], workdir)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("ERROR!!!") == 1 and msg in r.stdout


@needs_mpiexec
def test_mpiexec_missing_input_every_rank_exits_zero(workdir):
    r = mpirun("rowwise", 2, [6, 6], workdir)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("Unable to locate matrix file 'matrix_6_6.txt'") == 1
    assert "comm_sz = 2\nmy_rank = 0\n" in r.stdout  # the banner reports the launcher's P
    assert (workdir / "data" / "out" / "rowwise.csv").read_text() == "n_rows, n_cols, n_processes, time\n"


@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("dist", ["shared", "send"])
@pytest.mark.parametrize("alg", ALGS)
def test_mpiexec_rank_mode_fixture_matches_reference(workdir, golden, alg, dist):
    # the one-GPU-per-rank path (MPI bootstrap, RCCL communicator from the broadcast unique id,
    # shared-window or root-send distribution, max-over-ranks timing) at P = 1, collectives forced
    yout = workdir / "y.txt"
    env = dict(MVG_RANK_MODE=1, MVG_ALWAYS_COLLECT=1, MVG_ITERS=5, MVG_Y_OUT=yout)
    if dist == "send":
        env["MVG_DIST"] = "send"
    r = mpirun(alg, 1, [4, 8], workdir, **env)
    assert r.returncode == 0, r.stderr
    assert "launch: 1 ranks, one GPU each" in r.stdout
    assert ("shared window" in r.stdout) == (dist == "shared")
    assert max_rel(np.loadtxt(yout), golden[f"fixture_4x8/{alg}/P1"]) <= 1e-12
    lines = (workdir / "data" / "out" / f"{alg}.csv").read_text().splitlines()
    assert re.fullmatch(r"4, 8, 1, \d+\.\d{6}", lines[1]), lines


@needs_mpiexec
@pytest.mark.gpu
def test_mpiexec_more_ranks_than_gpus_fails_cleanly(workdir):
    import torch

    n = torch.cuda.device_count() + 1
    r = mpirun("rowwise", n, [4 * n, 8], workdir, MVG_SYNTH=1, MVG_ITERS=1)
    assert r.returncode != 0
    assert f"{n} GPU(s) needed on this node" in r.stderr


# ---- more than one rank on a one-GPU machine: every rank on GPU 0 (MVG_SAME_DEVICE=1), RCCL
# over loopback sockets. The multi-rank code path (MPI bootstrap, shared-window and root-send
# distribution, ncclGather / ncclReduce / ncclCommSplit + two-level exchange) against the real
# reference's own y for the same P.
@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("alg,P,dist", [("rowwise", 2, "shared"), ("rowwise", 4, "send"), ("colwise", 3, "shared"),
                                        ("colwise", 4, "send"), ("blockwise", 4, "shared"), ("blockwise", 3, "send")])
def test_mpiexec_multi_rank_matches_reference(tmp_path, golden, alg, P, dist):
    (tmp_path / "data" / "out").mkdir(parents=True)
    yout = tmp_path / "y.txt"
    env = dict(MVG_SYNTH=1, MVG_SAME_DEVICE=1, MVG_ITERS=3, MVG_Y_OUT=yout)
    if dist == "send":
        env["MVG_DIST"] = "send"
    r = mpirun(alg, P, [480, 480], tmp_path, **env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert f"launch: {P} ranks" in r.stdout
    assert max_rel(np.loadtxt(yout), golden[f"sq_480/{alg}/P{P}"]) <= 1e-12
    lines = (tmp_path / "data" / "out" / f"{alg}.csv").read_text().splitlines()
    assert re.fullmatch(rf"480, 480, {P}, \d+\.\d{{6}}", lines[1]), lines


@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("alg,P", [("rowwise", 3), ("colwise", 4), ("colwise", 3), ("blockwise", 4),
                                   ("blockwise", 2)])
def test_mpiexec_exact_mode_writes_the_references_y_file(tmp_path, golden, alg, P):
    # MVG_EXACT=1: P ranks (all on GPU 0), bit-exact kernels and the reference's combine order;
    # the y file is then the reference's own y dump (oracle/ref_dump.h, "%.17g" per line) byte
    # for byte — the block split at grids of at most two columns, where its sum is deterministic
    (tmp_path / "data" / "out").mkdir(parents=True)
    yout = tmp_path / "y.txt"
    r = mpirun(alg, P, [480, 480], tmp_path, MVG_SYNTH=1, MVG_SAME_DEVICE=1, MVG_EXACT=1, MVG_ITERS=3,
               MVG_Y_OUT=yout)
    assert r.returncode == 0, r.stderr[-2000:]
    want = "".join("%.17g\n" % v for v in golden[f"sq_480/{alg}/P{P}"])
    assert yout.read_text() == want


@pytest.mark.gpu
def test_bench_two_ranks_one_device(tmp_path):
    """bench.py's N > 1 path (the driver's scaling runs) at N = 2 under torch.distributed.run,
    both ranks on GPU 0: one JSON line, whole-job bytes, end-to-end y equal to the device y."""
    import json
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MVG_SAME_DEVICE="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--e2e-iters", "1", "--config-steps", "2",
                        "--config-e2e", "5"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["R"] == 32768 and d["config"]["bytes_per_step"] == 2 * 2147745792
    assert "mean_s" in d["end_to_end"]["root_send"]  # shared may be skipped when /dev/shm is small
    assert d["sections_s"]["headline"] > 0 and d["budget"]["skipped"] == [] and d.get("truncated") is None
    cfg = {c["config"]: c for c in d["configs"]}
    assert cfg["config 3"]["shard"] == [65536, 32768] and cfg["config 3"]["value"] > 0
    assert cfg["config 4"]["grid"] == [1, 2] and cfg["config 4"]["shard"] == [131072, 65536]
    assert cfg["config 5"]["shard"] == [2097152, 512] and cfg["config 5"]["value"] > 0
    # every config's y against the real reference's own rows at P = 2 (tests/golden/config_slices.npz)
    for name in ("config 3", "config 4"):
        ref = cfg[name]["reference_rows"]
        assert ref["P"] == 2 and ref["rows"] == 512 and ref["max_rel"] <= 1e-12, ref
        assert ref["exact_bit_identical"], ref  # grids of <= 2 columns: deterministic reference sums
    # the weak-scaled main workload's first rows are config 2's: against the reference's rows too
    assert d["reference_rows"]["max_rel"] <= 1e-12 and d["reference_rows"]["exact_bit_identical"], d["reference_rows"]
    # the transports RCCL reported for its connections (loopback sockets here: both ranks on GPU 0)
    assert d["rccl"]["logged"] and 2 in d["rccl"]["comm_sizes"] and d["rccl"]["transport_counts"], d["rccl"]


# ---- the drop-in contract at 1 GiB: the reference's text format written for a 16384 x 8192
# matrix (0.95 GB), read by the executables' parallel loader, four ranks under mpiexec (every
# rank on GPU 0), y against the real reference's own y for the same P.
@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("alg,R,C", [("rowwise", 16384, 8192), ("colwise", 8192, 16384), ("blockwise", 16384, 8192)])
def test_mpiexec_1gib_text_matches_reference(tmp_path, golden, alg, R, C):
    from matvec_mpi_multiplier_amd import multiplier as mm

    data = tmp_path / "data"
    (data / "out").mkdir(parents=True)
    mm.write_matr_synth(str(data / f"matrix_{R}_{C}.txt"), R, C, 42)
    mm.write_vec(str(data / f"vector_{C}.txt"), mm.synth_host(1, C, 4242)[0])
    yout = tmp_path / "y.txt"
    r = mpirun(alg, 4, [R, C], tmp_path, MVG_SAME_DEVICE=1, MVG_ITERS=2, MVG_Y_OUT=yout)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Reading matrix from file" in r.stdout
    name = f"big_{R}x{C}"
    assert max_rel(np.loadtxt(yout), golden[f"{name}/{alg}/P4"]) <= 1e-12


# ---- BASELINE.json config 1 as stated: the reference's fixture under `mpirun -np 2`
# (test.sh:11), every algorithm, through the drop-in executables (both ranks on GPU 0 here)
@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("alg", ALGS)
def test_config1_fixture_mpiexec_two_ranks(workdir, golden, alg, exact):
    yout = workdir / "y.txt"
    env = dict(MVG_SAME_DEVICE=1, MVG_ITERS=3, MVG_Y_OUT=yout)
    if exact:
        env["MVG_EXACT"] = 1
    r = mpirun(alg, 2, [4, 8], workdir, **env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "comm_sz = 2\nmy_rank = 0\n" in r.stdout and "launch: 2 ranks" in r.stdout
    want = golden[f"fixture_4x8/{alg}/P2"]
    if exact:  # the reference's own y dump, byte for byte
        assert yout.read_text() == "".join("%.17g\n" % v for v in want)
    else:
        assert max_rel(np.loadtxt(yout), want) <= 1e-12
    lines = (workdir / "data" / "out" / f"{alg}.csv").read_text().splitlines()
    assert re.fullmatch(r"4, 8, 2, \d+\.\d{6}", lines[1]), lines


# ---- eight ranks: the column split's 8 strips and the block split's 2 x 4 grid (config 4's
# grid, utils.c:26-37; grid-row ncclReduce over 4 ranks, then the leaders' ncclGather through
# ncclCommSplit), against the real reference's y at P = 8
@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("alg,case,R,C,exact", [
    ("colwise", "sq_480", 480, 480, False), ("colwise", "sq_480", 480, 480, True),
    ("blockwise", "sq_480", 480, 480, False), ("blockwise", "sq_480", 480, 480, True),
    ("colwise", "fixture_4x8", 4, 8, True), ("blockwise", "fixture_4x8", 4, 8, True),
])
def test_mpiexec_eight_ranks_match_reference(workdir, golden, alg, case, R, C, exact):
    from oracle import oracle

    yout = workdir / "y.txt"
    env = dict(MVG_SAME_DEVICE=1, MVG_ITERS=2, MVG_Y_OUT=yout)
    if case != "fixture_4x8":
        env["MVG_SYNTH"] = 1
    if exact:
        env["MVG_EXACT"] = 1
    r = mpirun(alg, 8, [R, C], workdir, **env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "launch: 8 ranks" in r.stdout
    if alg == "blockwise":
        assert "comm_sz_rows = 2\ncomm_sz_cols = 4\n" in r.stdout
    want = golden[f"{case}/{alg}/P8"]
    y = np.loadtxt(yout, ndmin=1)
    assert max_rel(y, want) <= 1e-12
    if exact and alg == "colwise":  # MPICH's reduce order, the reference's own y file
        assert yout.read_text() == "".join("%.17g\n" % v for v in want)
    elif exact:  # 2 x 4 grid: the reference adds in arrival order; the exact mode in rank order
        if case == "fixture_4x8":
            A = np.loadtxt(os.path.join(GOLDEN_DIR, "matrix_4_8.txt")).reshape(4, 8)
            x = np.loadtxt(os.path.join(GOLDEN_DIR, "vector_8.txt"))
        else:
            A, x = oracle.synth(R, C, 42), oracle.synth(1, C, 4242)[0]
        np.testing.assert_array_equal(y, oracle.multiply(alg, A, x, 8))


# ---- the column split at P = 5 and 10 on 720^2: MPICH's reduce-scatter + gather order for a
# y of more than 2 KiB, where it differs from a binomial tree (oracle/cpu_ref.c ref_mpich_reduce)
@needs_mpiexec
@pytest.mark.gpu
@pytest.mark.parametrize("P", [5, 10])
def test_mpiexec_exact_colwise_mpich_reduce_order(tmp_path, golden, P):
    (tmp_path / "data" / "out").mkdir(parents=True)
    yout = tmp_path / "y.txt"
    r = mpirun("colwise", P, [720, 720], tmp_path, MVG_SYNTH=1, MVG_SAME_DEVICE=1, MVG_EXACT=1, MVG_ITERS=2,
               MVG_Y_OUT=yout)
    assert r.returncode == 0, r.stderr[-2000:]
    assert yout.read_text() == "".join("%.17g\n" % v for v in golden[f"sq_720/colwise/P{P}"])


@pytest.mark.gpu
def test_bench_sigterm_mid_run_keeps_the_line(tmp_path):
    """The driver's N = 1 command terminated by a time limit while a GPU section runs: rank 0's
    watcher writes the line so far (headline included, `truncated`, the section it was in) and
    the process exits 128 + SIGTERM; sections that finished are in the line."""
    import json
    import signal
    import threading
    import time

    p = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "5", "--warmup", "2",
                          "--no-cpu-baseline", "--configs", "3,4", "--config-e2e", "4"],
                         cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    seen = threading.Event()
    err = []

    def watch():
        for ln in p.stderr:
            err.append(ln)
            if "section config 4 (estimate" in ln:  # config 4's 128 GiB shard, then its 137 GB end to end
                seen.set()

    t = threading.Thread(target=watch, daemon=True)
    t.start()
    try:
        assert seen.wait(timeout=100), "".join(err[-20:])
        time.sleep(1)  # inside config 4 (its fill, steps or the end-to-end host matrix)
        p.send_signal(signal.SIGTERM)
        out = p.stdout.read()
        assert p.wait(timeout=60) == 128 + signal.SIGTERM
    finally:
        if p.poll() is None:
            p.kill()
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    assert d["truncated"] is True and d["truncated_by"] == "SIGTERM" and d["truncated_in"].startswith("config 4")
    assert d["value"] > 0 and d["roofline"]["frac"] > 0 and d["exact"]["value"] > 0
    assert [c["config"] for c in d["configs"]] == ["config 3"]  # config 4 had not finished
    assert "headline" in d["sections_s"] and "config 3" in d["sections_s"]
