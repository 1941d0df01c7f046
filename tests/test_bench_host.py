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
    command's exit code, with no JSON line on stdout."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
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
                    "print('device-resident: 0.0500 ms per multiply, 123.4 GB/s aggregate; GEMV kernel 0.040 ms (max over GPUs)')\n")
    fake.chmod(0o755)

    class A:
        alg = "colwise"
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("NCCL_DEBUG", "INFO")  # what the bench sets for its own ranks
    r = bench.single_process_section(A(), 8, R, C, {"NCCL_DEBUG": "WARN", "NCCL_DEBUG_FILE": None}, exe=str(fake))
    assert r["ran"] and r["rc"] == 0, r
    assert r["ms_per_step"] == 0.05 and r["value"] == 123.4 and r["kernel_ms"] == 0.04 and r["end_to_end_s"] == 0.0001
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
    assert bench.kernel_family("hopxl_l8_w2_u16_n4") == "gemv_seq_hop_xl"
    assert bench.kernel_family("seqx_r64_t16_b2_g8") == "gemv_seq_x"
    assert bench.kernel_family("panel_l8_w2_u16 (column panels, P = 256)") == "gemv_seq_hop_panel"
    assert bench.kernel_family("rowlines_w8_u4_x0") == "gemv_rowblock_lines"


def test_pmc_summary_finds_the_committed_counters():
    """The headline roofline's `traffic`, `valu_busy` and `l2_hit` come from the committed PMC
    summaries (profiles/r04/pmc_<family>_<M>x<K>.json, tools/pmc_traffic.py)."""
    d = bench.pmc_summary(16384, 16384, "rowblk_w4_r2_u8")
    assert d is not None and d["source"].startswith("profiles/")
    assert 0.99 < d["traffic_over_algorithmic"] < 1.01
    assert 0.0 < d["valu_busy"] < 1.0 and 0.0 < d["l2_hit"] < 1.0
    assert bench.pmc_summary(16384, 16384, "panel_l8_w2_u16 (column panels, P = 256)")["source"].endswith(
        "pmc_gemv_seq_hop_panel_16384x16384.json")
    assert bench.pmc_summary(3, 5, "rowblk_w4_r2_u8") is None


def test_warm_runs_about_the_requested_time():
    """warm(): at least `min_launches`, then enough more for ~`seconds` of multiplies."""
    import time

    class Eng:
        calls = 0

        def multiply(self):
            Eng.calls += 1
            time.sleep(0.001)

        def sync(self):
            pass

    bench.warm(Eng(), 3, False, 0, seconds=0.03)
    assert 3 <= Eng.calls and 20 <= Eng.calls <= 40, Eng.calls
    Eng.calls = 0
    bench.warm(Eng(), 5, False, 0, seconds=0.0)
    assert Eng.calls == 5


def test_ref_sweep_reports_speedup_and_efficiency(monkeypatch):
    """cpu_baseline.sweep: S = T1 / TP and E = S / P (the reference's README.md:47-50), points that
    do not split the sample skipped, a failing point recorded."""
    from oracle import ref_runner

    secs = {1: 0.050, 2: 0.030, 4: 0.020, 8: 0.025}

    def fake_run(alg, R, C, p, timeout=None, cpus=None, rows=None):
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
