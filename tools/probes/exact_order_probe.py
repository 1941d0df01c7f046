"""The bench's exact section in both orders (development tool): the row-major exact kernel's
time inside the engine (config 2, MVG_NO_PANELS=1) measured before and after the panel copy was
built, used and freed, and the tree kernel around them.

    python tools/probes/exact_order_probe.py [rm-first|panels-first]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402


def run(eng, n=100, every=1):
    for _ in range(5):
        eng.multiply()
    eng.sync()
    eng.kernel_timing(every)
    for _ in range(n):
        eng.multiply()
    eng.sync()
    ms = eng.kernel_ms().avg_ms
    eng.kernel_timing(0)
    return round(ms * 1e3, 1)


def main():
    order = sys.argv[1] if len(sys.argv) > 1 else "panels-first"
    comm = mm.Comm.init_all([0])
    eng = mm.Multiplier("rowwise", 16384, 16384, comm)
    eng.fill_synth()
    eng.sync()
    out = {"order": order, "tree_0": run(eng)}

    def rm():
        os.environ["MVG_NO_PANELS"] = "1"
        eng.set_exact(True)
        r = run(eng)
        eng.set_exact(False)
        del os.environ["MVG_NO_PANELS"]
        return r

    def panels():
        eng.set_exact(True)
        r = run(eng)
        eng.set_exact(False)
        return r

    steps = [("rm", rm), ("panels", panels)] if order == "rm-first" else [("panels", panels), ("rm", rm)]
    for i in range(2):
        for name, fn in steps:
            out[f"{name}_{i}"] = fn()
        out[f"tree_{i + 1}"] = run(eng)
    print(json.dumps(out), flush=True)
    eng.destroy()
    comm.destroy()


if __name__ == "__main__":
    main()
