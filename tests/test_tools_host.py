"""The evidence tools on synthetic inputs (no GPU): tools/headline_launches.py picks the bench
headline's K timed launches out of a rocprofv3 kernel trace."""
import csv
import json
import os
import subprocess
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import headline_launches  # noqa: E402


def write_trace(path, rows):
    cols = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        for name, s, e, grid in rows:
            w.writerow([name, s, e, grid, 1, 1])


def bench_like_trace():
    """A fill, 150 tree launches (settle + warm-up + timed) with an RCCL kernel among them, the
    exact section's kernel, then more tree launches (a later config) — in shuffled file order."""
    rows = [("fill", i * 10, i * 10 + 5, 1) for i in range(3)]
    t = 1000
    for i in range(150):
        dur = 300_000 if i < 130 else 290_000 + i  # the last 20: 290.130 .. 290.149 us
        rows.append(("gemv_rowblock", t, t + dur, 2097152))
        t += dur + 1000
        if i == 60:
            rows.append(("ncclDevKernel_Gather", t, t + 500, 64))
            t += 1000
    rows.append(("gemv_seq_hop_n8", t, t + 400_000, 4096))
    t += 500_000
    rows += [("gemv_rowblock", t + i * 400_000, t + i * 400_000 + 350_000, 2097152) for i in range(200)]
    return rows


def test_headline_is_the_last_k_of_the_first_long_run():
    rows = sorted((s, e, name, grid) for name, s, e, grid in bench_like_trace())
    sel = headline_launches.headline(rows, 20)
    assert len(sel) == 20
    assert [round((e - s) / 1e3, 3) for s, e, _, _ in sel] == [round(290 + (130 + i) / 1e3, 3) for i in range(20)]
    assert headline_launches.headline(rows[:50], 20) == []  # no run long enough


def test_headline_cli(tmp_path):
    rows = bench_like_trace()
    write_trace(tmp_path / "run_kernel_trace.csv", rows[::-1])
    line = tmp_path / "bench.json"
    line.write_text(json.dumps({"metric": "m", "value": 7000.0, "roofline": {"kernel_ms": 0.29015}}) + "\n")
    out = tmp_path / "hl.json"
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "headline_launches.py"), str(tmp_path),
                        "--bench", str(line), "--out", str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["kernel"] == "gemv_rowblock" and d["grid_threads"] == 2097152
    assert len(d["launch_us"]) == 20 and abs(d["mean_us"] - 290.1395) < 1e-3
    assert d["line_kernel_us"] == 290.15 and d["line_value"] == 7000.0
