"""How the engine's HIP-event kernel timing compares with back-to-back wall time for the tree
and the row-major exact GEMV at config 2 (development probe; one JSON line per form).

    python tools/probes/event_timing_probe.py [M] [K] [steps] [forms] [torch]

forms: "tree,exact" (default) or one of them. torch: what PyTorch does in the process before the
engine exists — "none" (its GPU side unused; the package imports it before loading the library
since round 5, MVG_NO_TORCH=1 keeps it out), "set" (torch.cuda.set_device), "sync" (also
torch.cuda.synchronize: PyTorch's own HIP runtime — a second one, with its own HSA runtime, in
the wheel — comes up on the device), "ops" (also a device tensor, a page-locked host tensor and
a copy on a side stream, as the bench's PCIe probe); "late": set + sync after the engine exists.

For each form: a warm-up, then `steps` multiplies timed by events on every launch
(kernel_timing(1)), the same with every 5th launch (the bench's setting), and 3 * steps
multiplies back to back timed by the wall clock between device syncs (no events at all). Run it
under `rocprofv3 --kernel-trace` to set the per-launch durations beside these.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if os.environ.get("PROBE_TORCH_FIRST") == "1":  # PyTorch's libraries loaded before the library's
    import torch  # noqa: F401
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    forms = (sys.argv[4] if len(sys.argv) > 4 else "tree,exact").split(",")
    mode = sys.argv[5] if len(sys.argv) > 5 else "none"
    if mode not in ("none", "late"):
        import torch

        torch.cuda.set_device(0)
        if mode != "set":
            torch.cuda.synchronize()
        if mode == "ops":
            d = torch.ones(1 << 20, dtype=torch.float64, device="cuda:0")
            h = torch.empty(1 << 20, dtype=torch.float64, pin_memory=True)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
    os.environ["MVG_NO_PANELS"] = "1"  # the exact form a fresh distribution runs (row-major)
    comm = mm.Comm.init_all([0])
    eng = mm.Multiplier("rowwise", M, K, comm)
    eng.fill_synth()
    if mode == "late":  # PyTorch's runtime comes up after the library's (the bench's order)
        import torch

        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    nbytes = 8 * (M * K + K + M)
    try:
        for form in forms:
            eng.set_exact(form == "exact")
            for _ in range(300):
                eng.multiply()
            eng.sync()
            out = {"form": form, "torch": mode, "M": M, "K": K, "steps": steps}
            for every in (1, 5):
                eng.kernel_timing(every)
                for _ in range(steps):
                    eng.multiply()
                eng.sync()
                out[f"events_every_{every}_us"] = round(eng.kernel_ms().avg_ms * 1e3, 2)
                eng.kernel_timing(0)
            eng.sync()
            t0 = time.perf_counter()
            for _ in range(3 * steps):
                eng.multiply()
            eng.sync()
            out["wall_per_step_us"] = round((time.perf_counter() - t0) / (3 * steps) * 1e6, 2)
            out["wall_frac"] = round(nbytes / (out["wall_per_step_us"] * 1e-6) / 8e12, 4)
            print(json.dumps(out), flush=True)
    finally:
        eng.destroy()
        comm.destroy()


if __name__ == "__main__":
    main()
