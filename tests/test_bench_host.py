"""bench.py's host-side helpers on the CPU (no GPU): the RCCL transport report parser, the
reference-row check every config's y goes through, the launcher relay that lets `bench.py --gpus N`
run without torch.distributed.run, the check recorder, the PMC summary lookup, the warm-up and
the reference rank sweep."""
import json
import os
import subprocess
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
    # the WARN / ERROR lines are passed on to stderr (a caller's NCCL_DEBUG=WARN loses nothing)
    warn = "host:1234:1240 [0] NCCL WARN NET/Socket : message truncated"
    assert bench.rccl_warnings(lines + [warn + "\n"]) == [warn]


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
    # a y off by more than the bar is a failed check: recorded (the run then exits 1), not raised
    y[rows[0]] *= 1 + 1e-10
    bench.FAILURES.clear()
    bench.reference_rows_check(cfg_name, alg, R, C, n, y, None)
    assert len(bench.FAILURES) == 1 and "reference's own y" in bench.FAILURES[0]
    bench.FAILURES.clear()
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


def test_expect_records_failures_and_returns_the_condition():
    bench.FAILURES.clear()
    assert bench.expect(True, "fine") is True and bench.FAILURES == []
    assert bench.expect(False, "y differs") is False and bench.FAILURES == ["y differs"]
    bench.FAILURES.clear()


def test_launcher_cmd_is_the_drivers_n_gpu_command():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    assert cmd[-4:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "5"][-4:]
    assert cmd[-5] == os.path.join(REPO, "bench.py")
    assert 1024 <= bench.free_port() < 65536


def _child(code):
    return [sys.executable, "-c", code]


def test_relay_prints_rank0_line_and_passes_the_exit_code(capsys):
    line = json.dumps({"metric": "m", "value": 1.0})
    rc = bench.relay(_child(f"print('RCCL banner'); print({line!r})"))
    out = capsys.readouterr()
    assert rc == 0 and out.out.strip() == line and "RCCL banner" in out.err
    # a failing child: its exit code, even after a line
    assert bench.relay(_child(f"import sys; print({line!r}); sys.exit(3)")) == 3
    # exit 0 without a line is a failure too
    assert bench.relay(_child("print('no json here')")) == 1


def test_relay_passes_a_termination_on_to_the_ranks(tmp_path):
    """A time limit that terminates `bench.py --gpus N` must end the ranks it started too."""
    import time

    marker = tmp_path / "child_pid"
    child_py, parent_py = tmp_path / "child.py", tmp_path / "parent.py"
    child_py.write_text(f"import os, time\nopen({str(marker)!r}, 'w').write(str(os.getpid()))\ntime.sleep(60)\n")
    parent_py.write_text(f"import sys\nsys.path.insert(0, {REPO!r})\nimport bench\n"
                         f"bench.relay([sys.executable, {str(child_py)!r}])\n")
    p = subprocess.Popen([sys.executable, str(parent_py)])
    for _ in range(200):
        if marker.exists() and marker.read_text():
            break
        time.sleep(0.1)
    child = int(marker.read_text())
    p.terminate()
    assert p.wait(timeout=30) == 128 + 15
    for _ in range(50):  # the child is gone (reaped by the parent's wait)
        try:
            os.kill(child, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    else:
        raise AssertionError("the relayed child outlived its terminated parent")


def test_bench_without_launcher_starts_the_ranks_itself():
    """`python bench.py --gpus 2` with no WORLD_SIZE: bench.py runs torch.distributed.run itself as
    a child. Here (no GPU) the two ranks fail at their first GPU call, and that failure is the
    command's exit code; the only line on stdout is rank 0's line so far: no value, truncated by
    the error."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode != 0
    lines = r.stdout.strip().splitlines()
    assert len(lines) <= 1
    if lines:
        d = json.loads(lines[0])
        assert d["value"] is None and d["truncated"] is True and d["truncated_by"] == "error", d
    assert "torch.distributed" in r.stderr or "ChildFailedError" in r.stderr or "rank" in r.stderr.lower()


def test_single_process_section_needs_n_devices():
    class A:
        alg = "rowwise"
    r = bench.single_process_section(A(), 8, 8 * 16384, 16384)
    assert r["ran"] is False and "needs 8 devices" in r["why"]


def test_single_process_section_runs_the_executable_and_reads_its_line(tmp_path, monkeypatch):
    """With N devices visible, rank 0 runs the executables' one-process-N-GPU form as a child and
    records its device-resident line and y (here a stand-in executable on the CPU)."""
    import torch

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("MVG_SAME_DEVICE", raising=False)
    R, C = 64, 32
    fake = tmp_path / "multiplier_colwise"
    fake.write_text("#!/usr/bin/env python3\n"
                    "import os, sys\n"
                    "assert os.environ['MVG_NGPUS'] == '8' and os.environ['MVG_SYNTH'] == 'device'\n"
                    "assert 'RANK' not in os.environ and sys.argv[1:] == ['64', '32']\n"
                    "assert os.environ.get('NCCL_DEBUG') == 'WARN' and 'NCCL_DEBUG_FILE' not in os.environ\n"
                    "open(os.environ['MVG_Y_OUT'], 'w').write('1.5\\n' * 64)\n"
                    "print('end-to-end (multiply + y on root; inputs generated on the GPUs, nothing distributed): mean 0.000100 s over 50 iterations')\n"
                    "print('device-resident: 0.0500 ms per multiply, 123.4 GB/s aggregate; GEMV kernel 0.040 ms (max over GPUs)')\n"
                    "print('runtime: RCCL 22707 (/opt/rocm/lib/librccl.so.1), HIP 70226015 (/opt/rocm/lib/libamdhip64.so.7)')\n")
    fake.chmod(0o755)

    class A:
        alg = "colwise"
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("NCCL_DEBUG", "INFO")  # what the bench sets for its own ranks
    r = bench.single_process_section(A(), 8, R, C, {"NCCL_DEBUG": "WARN", "NCCL_DEBUG_FILE": None}, exe=str(fake))
    assert r["ran"] and r["rc"] == 0, r
    assert r["ms_per_step"] == 0.05 and r["value"] == 123.4 and r["kernel_ms"] == 0.04 and r["end_to_end_s"] == 0.0001
    assert r["runtime"]["rccl_version"] == "2.27.7" and r["runtime"]["rccl_origin"] == "rocm"
    assert "reference_rows" not in r  # the column split's config-2 rows are not the weak-scaled row split's
    # a failing executable is recorded, never raised and not counted as a failed check (the
    # scaling line's exit code stays 0); a wrong y from a run that finished is counted
    bad = tmp_path / "bad"
    bad.write_text("#!/bin/sh\necho boom >&2\nexit 3\n")
    bad.chmod(0o755)
    bench.FAILURES.clear()
    r = bench.single_process_section(A(), 8, R, C, None, exe=str(bad))
    assert r["rc"] == 3 and "boom" in r["error"] and bench.FAILURES == []
    short = tmp_path / "multiplier_short"
    short.write_text(fake.read_text().replace("* 64", "* 63"))
    short.chmod(0o755)
    r = bench.single_process_section(A(), 8, R, C, {"NCCL_DEBUG": "WARN", "NCCL_DEBUG_FILE": None}, exe=str(short))
    assert r["rc"] == 0 and len(bench.FAILURES) == 1 and "63" in bench.FAILURES[0]
    bench.FAILURES.clear()


def test_kernel_family_names():
    assert bench.kernel_family("rowblk_w4_r2_u8") == "gemv_rowblock"
    assert bench.kernel_family("rowblk_w8_r2_u4_splitk") == "gemv_rowblock_split"
    assert bench.kernel_family("vec_l64_r1_u4_nt1_o5") == "gemv_vec"
    assert bench.kernel_family("hop8_l8_w2_u16") == "gemv_seq_hop"
    assert bench.kernel_family("hop8e_l8_w2_u16_n8") == "gemv_seq_hop_n8"  # not the one-wave form's counters
    assert bench.kernel_family("hopxl_l8_w2_u16_n4") == "gemv_seq_hop_xl"
    assert bench.kernel_family("seqx_r64_t16_b2_g8") == "gemv_seq_x"
    assert bench.kernel_family("panel_l8_w2_u16 (column panels, P = 256)") == "gemv_seq_hop_panel"
    assert bench.kernel_family("rowlines_w8_u4_x0") == "gemv_rowblock_lines"


def test_pmc_summary_finds_the_committed_counters():
    """The headline roofline's `traffic`, `valu_busy` and `l2_hit` come from the committed PMC
    summaries (profiles/r04/pmc_<family>_<M>x<K>.json, tools/pmc_traffic.py)."""
    d = bench.pmc_summary(16384, 16384, "rowblk_w4_r2_u8")
    assert d is not None and all(p.startswith("profiles/") for p in ([d["source"]] if isinstance(d["source"], str) else d["source"]))
    assert 0.99 < d["traffic_over_algorithmic"] < 1.01
    assert 0.0 < d["valu_busy"] < 1.0 and 0.0 < d["l2_hit"] < 1.0
    assert bench.pmc_summary(16384, 16384, "panel_l8_w2_u16 (column panels, P = 256)")["source"].endswith(
        "pmc_gemv_seq_hop_panel_16384x16384.json")
    assert bench.pmc_summary(3, 5, "rowblk_w4_r2_u8") is None


def test_warm_runs_about_the_requested_time(monkeypatch):
    """warm(): at least `min_launches`, then enough more for ~`seconds` of multiplies (a fake
    clock that advances 1 ms per multiply, so the count does not depend on the host's load)."""
    clock = [0.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: clock[0])

    class Eng:
        calls = 0

        def multiply(self):
            Eng.calls += 1
            clock[0] += 0.001

        def sync(self):
            pass

    bench.warm(Eng(), 3, False, 0, seconds=0.03)
    assert 29 <= Eng.calls <= 30, Eng.calls
    Eng.calls = 0
    bench.warm(Eng(), 5, False, 0, seconds=0.0)
    assert Eng.calls == 5
    Eng.calls = 0
    bench.warm(Eng(), 2, False, 0)  # the default: 0.3 s of load before a supplementary section
    assert 299 <= Eng.calls <= 300, Eng.calls  # int() of 0.3 / 0.001 in floating point


def test_ref_sweep_reports_speedup_and_efficiency(monkeypatch):
    """cpu_baseline.sweep: S = T1 / TP and E = S / P (the reference's README.md:47-50), points that
    do not split the sample skipped, a failing point recorded."""
    from oracle import ref_runner

    secs = {1: 0.050, 2: 0.030, 4: 0.020, 8: 0.025}

    def fake_run(alg, R, C, p, timeout=None, cpus=None, rows=None, track=None):
        if p == 8:
            raise RuntimeError("mpiexec failed")
        return {"seconds": secs[p], "y": None, "wall_s": 1.0}

    monkeypatch.setattr(ref_runner, "run", fake_run)

    class A:
        ref_timeout = 10.0
    out = bench.ref_sweep(A(), "rowwise", 1024, 16384, 16, 0.040, "compact", (1, 2, 4, 8, 3), 8 * 1024 * 16384)
    pts = {p["P"]: p for p in out["points"]}
    assert sorted(pts) == [1, 2, 4, 16]  # 3 does not split 1024 rows; 8 failed
    assert pts[1]["speedup"] == 1.0 and pts[2]["speedup"] == round(0.05 / 0.03, 3)
    assert pts[16]["efficiency"] == round(0.05 / 0.04 / 16, 3) and pts[16]["placement"] == "compact"
    assert out["errors"] and "P=8" in out["errors"][0]


# ---- the wall-time budget and the truncated line (a time limit must not lose the scaling line)

def test_budget_skips_a_section_that_does_not_fit_and_records_times():
    b = bench.Budget(limit_s=bench.Budget(0).used() + 5.0)  # about 5 s left
    ran = []
    assert b.run("quick", 0.5, lambda v: ran.append(v) or v, 7) == 7
    got = b.run("huge", 3600.0, lambda: ran.append("huge"))
    assert ran == [7] and got["skipped"] == "budget" and got["need_s"] == 3600.0 and 0 < got["left_s"] <= 5
    assert set(b.sections) == {"quick"} and b.skipped == ["huge"]
    rec = b.record()
    assert rec["skipped"] == ["huge"] and rec["limit_s"] == b.limit_s
    # nested sections name the innermost one in progress, then restore the outer one
    seen = []
    b.run("outer", 0.0, lambda: b.run("inner", 0.0, lambda: seen.append(b.current)) or seen.append(b.current))
    assert seen == ["inner", "outer"] and b.current is None


def _budget_rank(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 1 is short of time, rank 0 is not: both must skip (no rank left waiting)
        b = bench.Budget(1e6 if rank == 0 else 0.0, distributed=True, device="cpu")
        got = b.run("section", 1.0, lambda: "ran")
        out.put((rank, got if isinstance(got, str) else got["skipped"]))
    finally:
        dist.destroy_process_group()


def test_budget_decision_is_all_reduced_over_ranks():
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_budget_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: "budget", 1: "budget"}


def test_report_writes_one_line_with_sections_and_warnings(tmp_path):
    import io

    buf = io.StringIO()
    b = bench.Budget(1e6)
    r = bench.Report(buf, b)
    r.update({"metric": bench.METRIC, "value": 1.5})
    b.run("configs", 0.0, lambda: r.append("configs", {"config": "config 3"}))
    bench.WARNINGS.append("single_process: failed")
    try:
        assert r.write() is True and r.write() is False  # once only
    finally:
        bench.WARNINGS.clear()
    lines = buf.getvalue().splitlines()
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.5 and d["configs"] == [{"config": "config 3"}] and "configs" in d["sections_s"]
    assert d["warnings"] == ["single_process: failed"] and d["failures"] is None and "truncated" not in d


_BLOCKED_RANK0 = r'''
import ctypes, os, sys, time
sys.path.insert(0, {repo!r})
import bench
b = bench.Budget(1e6)
r = bench.Report(sys.stdout, b)
r.update({{"metric": bench.METRIC, "value": 7166.9}})
r.watch_signals()
r["exact"] = {{"value": 1.0}}
b.sections["headline"] = 0.3
def blocked():
    open({marker!r}, "w").write("in")
    t0 = time.time()
    while time.time() - t0 < 60:  # the main thread inside a C call (a signal only cuts one sleep short)
        ctypes.CDLL(None).sleep(60)
b.run("config 4 end_to_end", 0.0, blocked)
print("not reached")
'''


def _start_blocked(tmp_path, wrap_in_relay):
    child = tmp_path / "rank0.py"
    marker = tmp_path / "marker"
    child.write_text(_BLOCKED_RANK0.format(repo=REPO, marker=str(marker)))
    if wrap_in_relay:
        parent = tmp_path / "relay.py"
        parent.write_text(f"import sys\nsys.path.insert(0, {REPO!r})\nimport bench\n"
                          f"sys.exit(bench.relay([sys.executable, {str(child)!r}]))\n")
        cmd = [sys.executable, str(parent)]
    else:
        cmd = [sys.executable, str(child)]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    import time

    for _ in range(300):
        if marker.exists():
            break
        time.sleep(0.1)
    assert marker.exists(), p.communicate(timeout=5)
    return p


@pytest.mark.parametrize("wrap_in_relay", [False, True])
def test_sigterm_mid_section_writes_the_truncated_line(tmp_path, wrap_in_relay):
    """A SIGTERM while rank 0's main thread is blocked in a C call (a GPU copy, the oracle):
    the watcher thread still writes the line so far, marked truncated, and the process exits
    128 + 15. Through the launcher-free relay (`bench.py --gpus N`) the same line comes out."""
    import signal

    p = _start_blocked(tmp_path, wrap_in_relay)
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=60)
    assert p.returncode == 128 + signal.SIGTERM, err
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "not reached" not in out, out
    d = json.loads(lines[0])
    assert d["truncated"] is True and d["truncated_by"] == "SIGTERM"
    assert d["truncated_in"] == "config 4 end_to_end"
    assert d["value"] == 7166.9 and d["exact"] == {"value": 1.0} and d["sections_s"]["headline"] == 0.3


def test_host_rows_region_is_page_aligned_within_the_matrix():
    A = np.zeros((1000, 513))
    lo, n = bench.host_rows_region(A, 100, 300)
    base, end = A.ctypes.data, A.ctypes.data + A.nbytes
    assert lo % 4096 == 0 or lo == base
    assert base <= lo <= base + 100 * 513 * 8 and lo + n >= base + 300 * 513 * 8 and lo + n <= end
    assert (lo + n) % 4096 == 0 or lo + n == end


def test_host_memory_and_cache_probes():
    assert bench.host_mem_free() > 0
    c = bench.host_cache()
    if c is not None:  # sysfs exposes the L3 on this host
        assert c["l3_bytes"] >= c["l3_instance_bytes"] > 0 and c["l3_bytes_system"] >= c["l3_bytes"]
    class A:
        pass
    rows = bench.big_sample_rows(A(), "rowwise", 16384, 16384)
    assert 8 * rows * 16384 >= max(1 << 30, 2 * ((c or {}).get("l3_bytes_system") or 0)) and rows <= 16384


def test_section_estimates_grow_with_the_work():
    assert bench.est_e2e(137e9, 1, 3, False) > bench.est_e2e(2.1e9, 1, 3, False) > 4
    assert bench.est_e2e(17e9, 8, 3, True) > bench.est_e2e(17e9, 8, 3, False)
    class A:
        ref_rows, cpu_sample_bytes, cpu_seconds = 1024, 2.2e9, 12.0
    small = bench.est_cpu_baseline(A(), 16384, 16384)
    assert bench.est_cpu_baseline(A(), 16384, 16384, big_rows=8192) > small > 24


def test_e2e_memory_gate_follows_the_measured_memory(monkeypatch):
    """configs[].end_to_end runs wherever the host copy of A fits the memory measured at that
    moment (and the cap, less this process's RSS), 8 GiB + 5 % to spare; otherwise it says why."""
    monkeypatch.setattr(bench, "host_mem_free", lambda: 300 << 30)
    monkeypatch.setattr(bench, "process_rss", lambda: 2 << 30)
    ok, mem = bench.e2e_memory_fit(131072, 131072, False, 0, cap=250 << 30)  # config 4: 137 GB
    assert ok and mem["need_bytes"] == 8 * 131072 ** 2 and mem["host_free_bytes"] == 248 << 30
    ok, mem = bench.e2e_memory_fit(131072, 131072, False, 0, cap=140 << 30)
    assert not ok and mem["host_free_bytes"] == 138 << 30
    monkeypatch.setattr(bench, "host_mem_free", lambda: 100 << 30)
    assert bench.e2e_memory_fit(65536, 65536, False, 0)[0]  # config 3: 34 GB
    assert not bench.e2e_memory_fit(131072, 131072, False, 0)[0]


def test_an_uncaught_error_still_writes_the_line_so_far(tmp_path):
    """A section error that ends the run (fatal at N > 1) leaves the line so far, truncated,
    with the error, and the process fails."""
    child = tmp_path / "rank0.py"
    child.write_text(f"import sys\nsys.path.insert(0, {REPO!r})\nimport bench\n"
                     "b = bench.Budget(1e6)\nr = bench.Report(sys.stdout, b)\n"
                     "r.update({'metric': bench.METRIC, 'value': 42.0})\nr.on_uncaught()\n"
                     "def boom():\n    raise MemoryError('hipHostRegister: out of memory')\n"
                     "b.run('config 4 end_to_end', 0.0, boom)\n")
    p = subprocess.run([sys.executable, str(child)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "MemoryError" in p.stderr
    (line,) = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(line)
    assert d["value"] == 42.0 and d["truncated"] is True and d["truncated_by"] == "error"
    assert d["truncated_in"] == "config 4 end_to_end" and d["error"].startswith("MemoryError")


def test_a_budget_skip_still_gives_one_line_with_the_marker(tmp_path):
    """A run whose budget runs out after the headline: the sections that no longer fit are
    skipped, each marked in its place, and the process still prints exactly one JSON line."""
    child = tmp_path / "rank0.py"
    child.write_text(f"import sys\nsys.path.insert(0, {REPO!r})\nimport bench\n"
                     "b = bench.Budget(b_used := bench.Budget(0).used() + 3.0)\n"
                     "r = bench.Report(sys.stdout, b)\n"
                     "r.update({'metric': bench.METRIC, 'value': 7184.6})\n"
                     "r['exact'] = b.run('exact', 0.5, lambda: {'value': 7000.0})\n"
                     "r['end_to_end'] = b.run('end_to_end', 600.0, lambda: {'mean_s': 0.04})\n"
                     "r['configs'] = [dict(config='config 4', **b.run('config 4', 900.0, lambda: {}))]\n"
                     "r.write()\n")
    p = subprocess.run([sys.executable, str(child)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    (line,) = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(line)
    assert d["value"] == 7184.6 and d["exact"] == {"value": 7000.0} and "truncated" not in d
    assert d["end_to_end"]["skipped"] == "budget" and d["end_to_end"]["need_s"] == 600.0
    assert d["configs"][0]["skipped"] == "budget"
    assert d["budget"]["skipped"] == ["end_to_end", "config 4"] and set(d["sections_s"]) == {"exact"}


def test_settle_runs_until_the_step_time_is_steady(monkeypatch):
    """settle(): bursts of multiplies for at least min_s (a fresh box's slow first phase is
    itself steady, so time must outlast it), then until three bursts agree, never longer than
    max_s (a fake clock: 4 ms per multiply during the slow phase, 2 ms after)."""
    clock = [0.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: clock[0])

    class Eng:
        def __init__(self, slow_s):
            self.t0 = clock[0]
            self.slow_s = slow_s
            self.calls = 0

        def multiply(self):
            self.calls += 1
            clock[0] += 0.004 if clock[0] - self.t0 < self.slow_s else 0.002

        def sync(self):
            pass

    e = Eng(0.3)
    r = bench.settle(e, 0.35, 5.0, False, 0, burst=5, tol=0.01)
    assert r["steady"] and 0.35 <= r["s"] < 0.4 and r["first_us_per_step"] == 4000.0
    assert r["last_us_per_step"] == 2000.0 and e.calls == 5 * r["bursts"]
    assert r["trace_s_us"][0] == [0.02, 4000.0]
    r = bench.settle(Eng(10.0), 0.05, 0.2, False, 0, burst=5, tol=0.01)  # slow throughout: steady at once
    assert r["steady"] and 0.05 <= r["s"] < 0.08
    flip = Eng(0.0)
    flip.multiply = lambda: clock.__setitem__(0, clock[0] + (0.002 if flip.calls % 2 else 0.003)) or setattr(
        flip, "calls", flip.calls + 1)
    r = bench.settle(flip, 0.05, 0.2, False, 0, burst=1, tol=1e-9)  # never steady: stops at max_s
    assert not r["steady"] and 0.2 <= r["s"] < 0.21


def test_config_order_puts_the_configs_defined_at_this_n_first():
    assert bench.config_order("auto", 8) == [5, 4, 3]  # all three are defined at 8 GPUs; 5 only there
    assert bench.config_order("auto", 1) == [3, 5, 4]  # config 3 (1/2/4/8) first, then smallest first
    assert bench.config_order("auto", 2) == [3, 5, 4] and bench.config_order("auto", 4) == [3, 5, 4]
    assert bench.config_order("4,3", 8) == [4, 3]  # an explicit list is kept as given


def _pass_args(**kw):
    import argparse

    a = argparse.Namespace(configs="auto", no_configs=False, config_e2e="3,4,5", no_e2e=False, e2e_iters=3,
                           no_cpu_baseline=False, no_config_cpu_baseline=False)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_config_passes_keep_every_device_resident_number_when_end_to_end_does_not_fit(capsys):
    """Round 5's N = 8 run with the driver's defaults lost config 5 to the /dev/shm setup of
    configs 3 and 4. Now every config's device-resident steps run before any end-to-end loop:
    with end-to-end estimates beyond the budget, every config still has its value and only
    end-to-end entries are skipped; the end-to-end loops that do run go smallest A first."""
    import io

    b = bench.Budget(limit_s=bench.Budget(0).used() + 15.0, verbose=False)
    rep = bench.Report(io.StringIO(), b)
    rep["configs"] = []
    calls = []
    by = {int(c[0].split()[-1]): c for c in bench.BASELINE_CONFIGS}

    def dev(k):
        calls.append(("device", k))
        got = b.run(by[k][0], 1.0, lambda: ({"config": by[k][0], "value": 100.0 + k}, np.full(4, float(k))))
        return got

    def e2e(k, y):
        calls.append(("e2e", k))
        assert y[0] == float(k)
        need = 8 * by[k][2] * by[k][3] / 0.8e9  # the round-5 /dev/shm rate: minutes
        return b.run(f"{by[k][0]} end_to_end", need, lambda: {"mean_s": 1.0})

    def head():
        calls.append(("e2e", "headline"))
        return b.run("end_to_end", 1.0, lambda: {"mean_s": 0.01})

    out = bench.config_passes(_pass_args(), 8, 0, b, rep, dev, e2e, lambda k, y: calls.append(("cpu", k)),
                              headline_e2e=head, headline_bytes=8 * 8 * 16384 * 16384)
    assert calls[:3] == [("device", 5), ("device", 4), ("device", 3)]
    # end-to-end smallest A first: headline (17.2 GB at N = 8) before config 5 (17.2 GB), 3 (34 GB), 4 (137 GB)
    assert calls[3:] == [("e2e", "headline"), ("e2e", 5), ("e2e", 3), ("e2e", 4)]
    line = rep.snapshot()
    assert [c["config"] for c in line["configs"]] == ["config 5", "config 4", "config 3"]
    assert all("value" in c for c in line["configs"])
    assert all(c["end_to_end"]["skipped"] == "budget" for c in line["configs"])
    assert line["end_to_end"] == {"mean_s": 0.01}
    assert set(b.skipped) == {"config 3 end_to_end", "config 4 end_to_end", "config 5 end_to_end"}
    assert set(out) == {3, 4, 5}


def test_config_passes_at_one_gpu_runs_the_cpu_baselines_last():
    import io

    b = bench.Budget(1e6, verbose=False)
    rep = bench.Report(io.StringIO(), b)
    rep["configs"] = []
    calls = []

    def dev(k):
        calls.append(("device", k))
        if k == 4:  # a config that does not fit in HBM: no later pass for it
            return {"config": "config 4", "skipped": "needs 140 GiB of HBM per GPU"}, None
        return {"config": f"config {k}", "value": 1.0}, np.zeros(2)

    bench.config_passes(_pass_args(config_e2e="3"), 1, 0, b, rep, dev,
                        lambda k, y: calls.append(("e2e", k)) or {"mean_s": 2.0},
                        lambda k, y: calls.append(("cpu", k)) or {"value": 4.2}, headline_e2e=None)
    assert calls == [("device", 3), ("device", 5), ("device", 4), ("e2e", 3), ("cpu", 3), ("cpu", 5)]
    cfg = {c["config"]: c for c in rep.snapshot()["configs"]}
    assert cfg["config 3"]["end_to_end"] == {"mean_s": 2.0} and cfg["config 3"]["cpu_baseline"] == {"value": 4.2}
    assert cfg["config 5"]["end_to_end"].startswith("not requested") and "end_to_end" not in cfg["config 4"]
    # the other ranks (N > 1) run the same device and end-to-end passes, never the CPU baselines
    calls.clear()
    bench.config_passes(_pass_args(config_e2e="3"), 2, 1, b, rep, dev,
                        lambda k, y: calls.append(("e2e", k)) or {}, lambda k, y: calls.append(("cpu", k)))
    assert calls == [("device", 3), ("device", 5), ("device", 4), ("e2e", 3)]


def test_parse_runtime_line_of_the_executables():
    out = ("device-resident: 0.0500 ms per multiply, 123.4 GB/s aggregate; GEMV kernel 0.040 ms (max over GPUs)\n"
           "runtime: RCCL 22707 (/opt/rocm/lib/librccl.so.1), HIP 70226015 (/opt/rocm/lib/libamdhip64.so.7)\n")
    r = bench.parse_runtime_line(out)
    assert r["rccl_version"] == "2.27.7" and r["rccl_origin"] == "rocm" and r["hip_runtime_version"] == 70226015
    assert r["hip_path"] == "/opt/rocm/lib/libamdhip64.so.7"
    assert bench.parse_runtime_line("no such line") is None


def test_host_setup_record_rates_follow_the_slowest_rank():
    rec = bench.host_setup_record({"rows": 100, "threads": 4, "fill_s": 0.5, "pin_bytes": 8e8, "pin_s": 0.2}, False, 1000)
    assert rec["fill_GBps"] == round(8 * 100 * 1000 / 0.5 / 1e9, 2) and rec["pin_GBps"] == 4.0
    assert rec["by_rank"][0]["threads"] == 4


def test_fill_threads_split_the_quota_over_local_ranks():
    from matvec_mpi_multiplier_amd.hostshare import fill_threads

    one = fill_threads(1)
    assert one >= 1 and fill_threads(8) == max(1, one // 8) and fill_threads(10 ** 6) == 1


def test_stop_children_ends_a_running_child_group():
    """A SIGTERM to the bench ends its children too (the watcher calls stop_children): a child
    started by run_child, with a grandchild in its session, is gone within the grace period."""
    import threading
    import time

    got = {}
    t = threading.Thread(target=lambda: got.update(r=bench.run_child(["sh", "-c", "sleep 60 & wait"], 120)))
    t0 = time.perf_counter()
    t.start()
    for _ in range(100):
        if bench.CHILDREN:
            break
        time.sleep(0.05)
    assert bench.CHILDREN
    bench.stop_children(grace_s=5.0)
    t.join(timeout=10)
    assert not t.is_alive() and got["r"].returncode != 0 and time.perf_counter() - t0 < 10
    assert not bench.CHILDREN


def test_timing_note_names_the_measurement():
    assert bench.timing_note(-1, 20).startswith("span:") and "/ 20 launches" in bench.timing_note(-1, 20)
    assert "every 5th" in bench.timing_note(5, 20)


def test_a_config_that_does_not_split_over_n_is_skipped_not_fatal():
    """At a GPU count a config does not divide over (config 3's 65536 columns over 3 GPUs) the
    config is recorded as skipped on every rank before any collective, as the reference prints
    its ERROR!!! instead of running."""
    import argparse

    from matvec_mpi_multiplier_amd import multiplier as mm

    entry, y = bench.config_device(argparse.Namespace(config_steps=20), mm, None, 3, 0, 0, False, None, None, None, 3)
    assert y is None and entry["config"] == "config 3" and entry["skipped"].startswith("does not split over 3 GPUs")


def test_wait_vram_cleared_waits_for_the_drivers_clearing(monkeypatch):
    """After a large free the driver still counts the memory as used while it clears it in the
    background (and HBM-bound kernels run slow meanwhile); the bench waits, untimed and bounded,
    until the driver's count is back to what this process holds (fake clock and counters)."""
    import torch

    clock = [0.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: clock[0])
    monkeypatch.setattr(bench.time, "sleep", lambda s: clock.__setitem__(0, clock[0] + s))
    monkeypatch.delenv("MVG_SAME_DEVICE", raising=False)
    GiB = 1 << 30
    own = 3 * GiB
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (288 * GiB - own, 288 * GiB))
    # 128 GiB pending until t = 3.9 s, then only this process's own memory
    monkeypatch.setattr(bench, "_sysfs_vram_used", lambda local: own + (128 * GiB if clock[0] < 3.9 else 0))
    r = bench.wait_vram_cleared(0)
    assert r["pending_gib"] == 128.0 and r["left_gib"] == 0.0 and 3.9 <= r["waited_s"] <= 4.0
    assert bench.wait_vram_cleared(0)["waited_s"] == 0.0  # nothing pending: no wait
    # a count that never moves is an offset, not clearing: bounded once, then not waited on
    monkeypatch.setattr(bench, "_VRAM_OFFSET", {})
    monkeypatch.setattr(bench, "_sysfs_vram_used", lambda local: own + 50 * GiB)
    r = bench.wait_vram_cleared(0, timeout_s=2.0)
    assert 2.0 <= r["waited_s"] < 2.1 and r["left_gib"] == 50.0 and r["offset_learned_gib"] == 50.0
    r = bench.wait_vram_cleared(0, timeout_s=2.0)
    assert r["waited_s"] == 0.0 and r["pending_gib"] == 0.0
    # clearing on top of the offset is still waited for
    t_free = clock[0]
    monkeypatch.setattr(bench, "_sysfs_vram_used", lambda local: own + 50 * GiB + (16 * GiB if clock[0] < t_free + 0.5 else 0))
    r = bench.wait_vram_cleared(0, timeout_s=2.0)
    assert r["pending_gib"] == 16.0 and 0.5 <= r["waited_s"] < 0.6 and "offset_learned_gib" not in r
    # no sysfs (or a same-device rehearsal): nothing to wait on
    monkeypatch.setattr(bench, "_sysfs_vram_used", lambda local: None)
    assert bench.wait_vram_cleared(0) is None
    monkeypatch.setenv("MVG_SAME_DEVICE", "1")
    assert bench.wait_vram_cleared(0) is None


def test_executable_runtime_names_the_executables_rccl():
    """The line's runtime.executables: the RCCL / HIP the drop-in executables bind (their
    MVG_RUNTIME_ONLY=1 line: /opt/rocm's, where the Python ranks run PyTorch's), no GPU needed."""
    r = bench.executable_runtime("rowwise")
    if r is None:
        pytest.skip("bin/multiplier_rowwise not built")
    assert r["rccl_origin"] == "rocm" and r["rccl_version"].count(".") == 2 and r["hip_origin"] == "rocm"
