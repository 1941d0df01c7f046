"""Shared test setup.

`-m "not gpu"` : oracle vs the reference's golden vectors, host logic (planner, exchange
                 schedule, text I/O), the C-ABI library's exports, multi-rank gloo replays.
`-m gpu`       : parity of the HIP path (through the C-ABI) against the oracle/golden data.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_DIR = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    lib = os.path.join(REPO, "matvec_mpi_multiplier_amd", "libmatvec_gpu.so")
    if not os.path.exists(lib) or not os.path.exists(os.path.join(REPO, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", REPO, "-j8"], check=True)


@pytest.fixture(scope="session")
def golden():
    """{"<case>/<alg>/P<p>": y} produced by the real reference (tests/golden/make_golden.py)."""
    with np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        return json.load(f)


def case_inputs(case: dict):
    """A, x of a golden case: the reference's own fixture files, or the synthetic spec."""
    from oracle import oracle

    if case["source"] == "fixture":
        A = np.loadtxt(os.path.join(GOLDEN_DIR, f"matrix_{case['R']}_{case['C']}.txt")).reshape(case["R"], case["C"])
        x = np.loadtxt(os.path.join(GOLDEN_DIR, f"vector_{case['C']}.txt")).reshape(case["C"])
        return A, x
    return oracle.synth(case["R"], case["C"], 42), oracle.synth(1, case["C"], 4242)[0]


def golden_runs(manifest):
    for case in manifest["cases"]:
        for alg, plist in case["runs"].items():
            for p in plist:
                yield case, alg, p


def max_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.size == 0:
        return 0.0
    den = np.maximum(np.abs(b), np.finfo(np.float64).tiny)
    return float(np.max(np.abs(a - b) / den))
