"""The row-major exact GEMV in different contexts (development tool, one MI355X): why does the
bench's `exact.row_major` read below the same kernel in a sweep?

    python tools/probes/exact_context_probe.py MODE [M] [K] [launches]

MODE
  engine    : the tree and exact kernels three ways in one process, interleaved twice — through
              the engine (mm.Multiplier, MVG_NO_PANELS=1, its own stream and HIP events), on
              buffers from the engine's allocator launched on the default stream, and on torch
              buffers (the sweeps' setup);
  sustained : every config-2 form (tree, row-major exact variants, the panel form) for `launches`
              back-to-back launches after 0.1 s of load, each launch bracketed by its own events,
              with the GPU's clock, power and temperature after (rocm-smi), two passes in opposite
              orders;
  queues    : the tree and the exact kernel on the default stream and on 8 fresh streams (HIP maps
              streams onto GPU_MAX_HW_QUEUES hardware queues round robin), interleaved twice;
  isolate   : the raw exact kernel on torch buffers and the default stream, timed in bursts before
              and after each step that builds up the engine's process state: two more HIP streams,
              a page-locked host buffer with copies on them, an RCCL-less engine (mm.Multiplier),
              its destruction (PROBE_EXACT_VARIANTS=a,b adds exact variants by name);
  repeat    : the tree and the row-major exact variants (default placement, and the evenly placed
              hop8e_* forms) timed 12 times each, interleaved, each time after 0.1 s of load: the
              spread of one kernel's time from one burst to the next.
One JSON line per measurement.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("MVG_NO_PANELS", "1")
from matvec_mpi_multiplier_amd import multiplier as mm  # noqa: E402
from matvec_mpi_multiplier_amd._lib import check, lib  # noqa: E402

DEV = torch.device("cuda:0")


def inputs(M, K, s):
    A = torch.empty(M * K, dtype=torch.float64, device=DEV)
    x = torch.empty(K, dtype=torch.float64, device=DEV)
    y = torch.empty(M, dtype=torch.float64, device=DEV)
    check(lib.mvg_synth_fill_device(A.data_ptr(), K, M, K, 0, 0, K, 42, s), "fill A")
    check(lib.mvg_synth_fill_device(x.data_ptr(), K, 1, K, 0, 0, K, 4242, s), "fill x")
    return A, x, y


def exact_variant(name):
    names = [lib.mvg_gemv_exact_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_variant_count())]
    return names.index(name)


def per_launch_us(f, n, stream=None):
    """`n` back-to-back launches of f, each between its own events: sorted durations (us)."""
    st = stream or torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(st)
        f()
        b.record(st)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showtemp", "--json"],
                           capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        return {k: v for k, v in card.items() if any(s in k.lower() for s in ("sclk", "power", "junction", "memory"))}
    except Exception as exc:  # informative only
        return {"error": str(exc)[:80]}


def mode_engine(M, K, n):
    def timed(fn):
        fn()
        torch.cuda.synchronize()
        us = per_launch_us(fn, n)
        return sorted(us)[n // 2]

    s = torch.cuda.current_stream().cuda_stream
    tA, tx, ty = inputs(M, K, s)
    ptrs = []
    for count in (M * K, K, M):
        p = C.c_void_p()
        check(lib.mvg_malloc(C.byref(p), count * 8), "mvg_malloc")
        ptrs.append(p.value)
    hA, hx, hy = ptrs
    check(lib.mvg_synth_fill_device(hA, K, M, K, 0, 0, K, 42, s), "fill")
    check(lib.mvg_synth_fill_device(hx, K, 1, K, 0, 0, K, 4242, s), "fill")
    comm = mm.Comm.init_all([0])
    eng = mm.Multiplier("rowwise", M, K, comm)
    eng.fill_synth()
    eng.sync()
    res = {}
    for _ in range(2):
        for way in ("engine", "hipmalloc", "torch"):
            out = {}
            if way == "engine":
                for exact in (False, True):
                    eng.set_exact(exact)
                    for _ in range(3):
                        eng.multiply()
                    eng.kernel_timing(1)
                    for _ in range(n):
                        eng.multiply()
                    out["exact" if exact else "tree"] = eng.kernel_ms().avg_ms * 1e3
                    eng.kernel_timing(0)
                eng.set_exact(False)
            else:
                A, x, y = (hA, hx, hy) if way == "hipmalloc" else (tA.data_ptr(), tx.data_ptr(), ty.data_ptr())
                out["tree"] = timed(lambda: lib.mvg_gemv(A, K, x, y, M, K, s))
                out["exact"] = timed(lambda: lib.mvg_gemv_exact(A, K, x, y, M, K, s))
            for k, v in out.items():
                res.setdefault((way, k), []).append(round(v, 2))
    for (way, k), v in res.items():
        print(json.dumps({"mode": "engine", "M": M, "K": K, "way": way, "kernel": k, "us": v}), flush=True)
    eng.destroy()
    comm.destroy()
    for p in ptrs:
        lib.mvg_free(p)


def mode_sustained(M, K, n):
    s = torch.cuda.current_stream().cuda_stream
    A, x, y = inputs(M, K, s)
    P = 256
    Ap = torch.empty(M * P * (-(-K // P)), dtype=torch.float64, device=DEV)
    check(lib.mvg_panel_relayout(A.data_ptr(), K, M, K, Ap.data_ptr(), M * P, P, s), "relayout")
    forms = ["tree", "hop8_l8_w2_u16", "hop8_l8_w2_u24", "seqx_r64_t16_b2_g8", "seqx_r32_t64_b2_g8", "panels"]

    def fn(form):
        if form == "tree":
            return lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)
        if form == "panels":
            return lambda: lib.mvg_gemv_exact_panels(Ap.data_ptr(), M * P, P, x.data_ptr(), y.data_ptr(), M, K, 0, s)
        v = exact_variant(form)
        return lambda: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)

    heat = fn("tree")
    for order in (forms, forms[::-1]):
        for form in order:
            f = fn(form)
            if f() != 0:
                continue
            torch.cuda.synchronize()
            for _ in range(int(0.1 / 300e-6)):
                heat()
            us = per_launch_us(f, n)
            srt, tenth = sorted(us), max(1, n // 10)
            print(json.dumps({"mode": "sustained", "M": M, "K": K, "form": form, "launches": n,
                              "median_us": round(srt[n // 2], 2), "p10_us": round(srt[n // 10], 2),
                              "p90_us": round(srt[9 * n // 10], 2),
                              "first_tenth_us": round(sorted(us[:tenth])[tenth // 2], 2),
                              "last_tenth_us": round(sorted(us[-tenth:])[tenth // 2], 2),
                              "smi_after": smi()}), flush=True)


def mode_queues(M, K, n, nstreams=8):
    s0 = torch.cuda.current_stream()
    A, x, y = inputs(M, K, s0.cuda_stream)
    streams = [("default", s0)] + [(f"stream{i}", torch.cuda.Stream(device=DEV)) for i in range(nstreams)]
    hop = exact_variant("hop8_l8_w2_u16")
    kernels = {
        "tree": lambda h: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, h),
        "exact_hop8": lambda h: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, hop, h),
    }
    res = {}
    for _ in range(2):
        for sname, st in streams:
            h = st.cuda_stream
            for kname, f in kernels.items():
                torch.cuda.synchronize()
                for _ in range(int(0.1 / 300e-6)):
                    kernels["tree"](h)
                us = sorted(per_launch_us(lambda: f(h), n, st))
                res.setdefault((sname, kname), []).append(round(us[n // 2], 2))
    for (sname, kname), v in res.items():
        print(json.dumps({"mode": "queues", "M": M, "K": K, "stream": sname, "kernel": kname, "median_us": v}),
              flush=True)


def mode_isolate(M, K, n, reps=4):
    s0 = torch.cuda.current_stream()
    s = s0.cuda_stream
    A, x, y = inputs(M, K, s)
    hop, hope = exact_variant("hop8_l8_w2_u16"), exact_variant("hop8e_l8_w2_u16_n8")
    exact = lambda: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, hop, s)  # noqa: E731
    even = lambda: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, hope, s)  # noqa: E731
    tree = lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)  # noqa: E731
    P = 256
    Ap = torch.empty(M * P * (-(-K // P)), dtype=torch.float64, device=DEV)
    check(lib.mvg_panel_relayout(A.data_ptr(), K, M, K, Ap.data_ptr(), M * P, P, s), "relayout")
    pnames = [lib.mvg_gemv_exact_panel_variant_name(v).decode() for v in range(lib.mvg_gemv_exact_panel_variant_count())]

    def panel(name):
        v = pnames.index(name)
        return lambda: lib.mvg_gemv_exact_panels(Ap.data_ptr(), M * P, P, x.data_ptr(), y.data_ptr(), M, K, v, s)

    kernels = [("tree", tree), ("exact_hop8", exact), ("exact_hop8e_n8", even)]
    for name in filter(None, os.environ.get("PROBE_EXACT_VARIANTS", "").split(",")):
        v = exact_variant(name)
        kernels.append((name, lambda v=v: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)))
    kernels += [(n, panel(n)) for n in ("panel_l8_w2_u8",) if n in pnames]

    def bursts(stage):
        for kname, f in kernels:
            meds = []
            for _ in range(reps):
                torch.cuda.synchronize()
                for _ in range(int(0.1 / 300e-6)):
                    tree()
                us = sorted(per_launch_us(f, n))
                meds.append(round(us[n // 2], 2))
            print(json.dumps({"mode": "isolate", "M": M, "K": K, "stage": stage, "kernel": kname,
                              "burst_medians_us": meds}), flush=True)

    bursts("fresh process")
    extra = [torch.cuda.Stream(device=DEV) for _ in range(2)]
    for st in extra:  # used once each, as the engine's streams are
        with torch.cuda.stream(st):
            torch.empty(1024, device=DEV).fill_(1.0)
    torch.cuda.synchronize()
    bursts("+ two used streams")
    h = torch.empty(1 << 19, dtype=torch.float64, pin_memory=True)
    d = torch.empty(1 << 19, dtype=torch.float64, device=DEV)
    for st in extra:
        with torch.cuda.stream(st):
            d.copy_(h, non_blocking=True)
            h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    bursts("+ page-locked copies on them")
    comm = mm.Comm.init_all([0])
    eng = mm.Multiplier("rowwise", M, K, comm)
    eng.fill_synth()
    eng.sync()
    bursts("+ an engine")
    eng.destroy()
    comm.destroy()
    torch.cuda.synchronize()
    bursts("engine destroyed")


def mode_repeat(M, K, n, reps=12):
    s = torch.cuda.current_stream().cuda_stream
    A, x, y = inputs(M, K, s)
    forms = ["tree", "hop8_l8_w2_u16", "hop8e_l8_w2_u16_n8", "hop8e_l8_w2_u16_n4"]

    def fn(form):
        if form == "tree":
            return lambda: lib.mvg_gemv(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, s)
        v = exact_variant(form)
        return lambda: lib.mvg_gemv_exact_variant(A.data_ptr(), K, x.data_ptr(), y.data_ptr(), M, K, v, s)

    res = {f: [] for f in forms}
    heat = fn("tree")
    for _ in range(reps):
        for form in forms:
            f = fn(form)
            torch.cuda.synchronize()
            for _ in range(int(0.1 / 300e-6)):
                heat()
            us = sorted(per_launch_us(f, n))
            res[form].append(round(us[n // 2], 2))
    for form, v in res.items():
        srt = sorted(v)
        print(json.dumps({"mode": "repeat", "M": M, "K": K, "form": form, "burst_medians_us": v,
                          "min_us": srt[0], "median_us": srt[len(srt) // 2], "max_us": srt[-1]}), flush=True)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "engine"
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    {"engine": mode_engine, "sustained": mode_sustained, "queues": mode_queues, "repeat": mode_repeat,
     "isolate": mode_isolate}[mode](M, K, n)


if __name__ == "__main__":
    main()
