"""Benchmark: device-resident distributed fp64 GEMV (BASELINE.json metric) on N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--alg rowwise|colwise|blockwise]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

Workload (BASELINE.json configs[1], weak-scaled): every GPU owns a 16384 x 16384 fp64 row
shard of a (16384*N) x 16384 matrix (N = 1: exactly config 2, "Square N=16384 fp64 row-split
on 1 MI355X"), inputs synthetic (include/matvec_gpu.h spec) and resident in HBM. One step =
one pass of the hot path: the HIP GEMV on every shard + the RCCL exchange (ncclGather of y
to rank 0). K steps are timed between barrier + device synchronize on both sides; the time
is the max over ranks; value = algorithmic bytes of all ranks / that time.

Also reported: `roofline` (the GEMV kernel alone: bytes per launch / its mean duration from
HIP events on the engine stream — at one rank one event pair spanning the timed GEMVs, at N > 1
every 5th step's GEMV bracketed; peak 8 TB/s; `traffic` from the committed rocprofv3 PMC
summary when one matches this configuration), `cpu_baseline` (rank 0 at N = 1: the real
reference, oracle/_ref under mpiexec, on a sample of the same matrix, with the oracle's
restatement of its MPI loop on the full matrix beside it; the restatement alone when the
reference cannot run; its value from a sample beyond the host's L3), `end_to_end` (distribution
from the root's host memory + multiply + y on the root, the reference's timing semantics; also
under every config whose A fits the host memory measured at run time), and `configs`:
BASELINE.json configs 3-5 at their
own fixed sizes on the same N GPUs (strong scaling, device-resident, same engine, same step),
so one scaling run covers every multi-GPU config (each also in bit-exact mode, `configs[].exact`);
supplementary, never `value`. Each config carries `reference_rows` (its y against the real
reference's own y on four bands of its rows at P = N, tests/golden/config_slices.npz) and, at
N = 1, a `cpu_baseline` of its own (the reference on a 512 MiB row slice, the -O2 port on the
whole config up to 35 GB). `exact`: the same workload with the engine in bit-exact mode
(mvg_engine_set_exact: y identical to the reference's sequential sums) — repeated multiplies on
the engine's column-panel copy, and `row_major`, the kernels a fresh distribution runs — its step
rate and kernel roofline fraction, and (rank 0, N = 1, row split) its y compared bit for bit with
the oracle port's and the real reference's. At N > 1: `rccl` (the transport RCCL chose for every
connection and the communicator sizes, from its NCCL_DEBUG=INFO log) and `kernel_ms_by_rank`.

Wall-time budget (--budget-s): the headline is timed first; every section after it first checks
that its estimated time fits in what is left of the budget (at N > 1 the decision is all-reduced,
so every rank skips the same sections) and is recorded as {"skipped": "budget", ...} when it does
not. `sections_s` holds each section's wall time. If rank 0 receives SIGTERM / SIGINT (a time
limit around the run) or an error ends the run, it writes the line it has so far, marked
"truncated": true, and exits. `warnings` lists product paths that ran and failed without failing
a check (the single-process executable at N > 1). Progress goes to stderr every 30 s.
"""
from __future__ import annotations

import argparse
import copy
import gc
import glob
import json
import os
import signal
import sys
import threading
import time

import numpy as np

T_START = time.perf_counter()  # the budget counts from here (imports included)

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

SHARD = 16384  # rows per GPU and columns (config 2)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "fp64 GEMV achieved HBM GB/s per GPU + end-to-end time at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--alg", default="rowwise", choices=["rowwise", "colwise", "blockwise"])
    ap.add_argument("--rows", type=int, default=None, help="global rows (default 16384*N)")
    ap.add_argument("--cols", type=int, default=SHARD)
    ap.add_argument("--e2e-iters", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=1.5,
                    help="untimed multiplies before the W warm-up steps, at least this long (a fresh box's slow "
                         "phase is itself steady, so time must outlast it) and until the per-step time is "
                         "steady (0: none)")
    ap.add_argument("--settle-max-s", type=float, default=10.0)
    ap.add_argument("--event-every", type=int, default=None,
                    help="kernel duration for the roofline: bracket every Nth step's GEMV with HIP events "
                         "(N > 0), or -1: one event pair spanning the timed steps' GEMVs (default -1 at one "
                         "rank: no marker between the steps; 5 at N > 1, where the GEMV stream also waits "
                         "on the exchange)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work")
    ap.add_argument("--cpu-sample-bytes", type=float, default=2.2e9,
                    help="CPU baseline runs on the leading rows of the same matrix up to this size")
    ap.add_argument("--no-ref-baseline", action="store_true",
                    help="time only the oracle port, not the real reference (oracle/_ref)")
    ap.add_argument("--ref-rows", type=int, default=1024,
                    help="rows of the sample the real reference runs on (its loop is 100 iterations)")
    ap.add_argument("--ref-timeout", type=float, default=240.0)
    ap.add_argument("--cpu-sweep", default="1,2,4,8",
                    help="rank counts the real reference also runs at on the headline sample (cpu_baseline.sweep), "
                         "besides the host's CPU quota; '' skips the sweep")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE configs 3-5 section")
    ap.add_argument("--configs", default="auto",
                    help="which BASELINE configs the section runs, in order; auto: those BASELINE.json defines at "
                         "this N first (N = 8: 5, 4, 3), then the rest smallest first (config_order)")
    ap.add_argument("--config-steps", type=int, default=20)
    ap.add_argument("--no-config-cpu-baseline", action="store_true",
                    help="skip the per-config CPU baselines (configs 3-5, N = 1)")
    ap.add_argument("--config-ref-bytes", type=float, default=512 * 2 ** 20,
                    help="size of the leading-row slice the real reference runs on per config (>= 128 rows; "
                         "512 MiB: twice the L3 of the 16 CPUs its ranks use on the MI355X boxes)")
    ap.add_argument("--config-cpu-sample-bytes", type=float, default=3.5e10,
                    help="the port runs a config whole up to this size (configs 3, 5), else its leading rows")
    ap.add_argument("--config-cpu-seconds", type=float, default=4.0)
    ap.add_argument("--config-e2e", default="3,4,5",
                    help="configs that also run the end-to-end loop, wherever host memory (and /dev/shm at "
                         "N > 1) holds their A, measured at run time; '' for none")
    ap.add_argument("--host-mem-cap-gib", type=float, default=250.0,
                    help="host memory the end-to-end loops may assume at most (the GPU pool caps a command near "
                         "270 GiB, which the cgroup may not show)")
    ap.add_argument("--budget-s", type=float, default=420.0,
                    help="wall-time budget of the whole run (about 70 %% of the driver's 600 s limit): a "
                         "section whose estimate no longer fits is skipped and marked")
    ap.add_argument("--no-multi", action="store_true", help="skip the multi-vector GEMV section")
    ap.add_argument("--no-loader", action="store_true", help="skip the text-loader section")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the bit-exact section (the same workload with mvg_engine_set_exact)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


FAILURES: list[str] = []  # the bench's parity checks that failed (JSON `failures`; exit code 1)
WARNINGS: list[str] = []  # product paths that ran and failed without failing a check (JSON `warnings`)
CHILDREN: set = set()  # live child processes (each the leader of its own session): ended with the run


def stop_children(grace_s: float = 5.0) -> None:
    """End every live child's process group (the single-process executable driving N GPUs, the
    reference under mpiexec): SIGTERM, then SIGKILL after `grace_s`. Called when a signal ends
    the run, so a supervisor that signals only this process leaves nothing running."""
    live = list(CHILDREN)
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
    t0 = time.perf_counter()
    for p in live:
        try:
            p.wait(timeout=max(0.1, grace_s - (time.perf_counter() - t0)))
        except Exception:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass


def run_child(cmd, timeout, **kw):
    """subprocess.run(capture_output, text) in a session of its own, registered in CHILDREN
    while it runs; its whole process group is killed at the time limit."""
    import subprocess

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True, **kw)
    CHILDREN.add(p)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.communicate()
        raise
    finally:
        CHILDREN.discard(p)
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


class Budget:
    """The run's wall-time budget, counted from the start of the process (T_START). `run(name,
    need_s, fn, ...)` runs a section only when its estimate fits in what is left — at N > 1 the
    answer is all-reduced (MIN), so every rank takes the same sections and no rank waits in a
    collective another one skipped — and records its wall time in `sections`; a section that does
    not fit returns a skip marker instead. `current` names the section in progress (a truncated
    line says where the run was)."""

    def __init__(self, limit_s: float, distributed: bool = False, device=None, verbose: bool = True,
                 reserve_s: float = 0.0):
        self.limit_s = float(limit_s)
        self.distributed = distributed
        self.device = device
        self.verbose = verbose      # section log lines (rank 0 only at N > 1)
        self.reserve_s = reserve_s  # kept back for the teardown and the line
        self.sections: dict[str, float] = {}
        self.skipped: list[str] = []
        self.current: str | None = None
        self.failed_in: str | None = None

    def used(self) -> float:
        return time.perf_counter() - T_START

    def left(self) -> float:
        return self.limit_s - self.used()

    def fits(self, need_s: float, collective: bool = True) -> bool:
        ok = self.left() - self.reserve_s >= need_s
        if self.distributed and collective:
            import torch
            import torch.distributed as dist

            t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = float(t[0]) >= 1.0
        return ok

    def marker(self, need_s: float) -> dict:
        return {"skipped": "budget", "need_s": round(need_s, 1), "left_s": round(self.left(), 1)}

    def run(self, name: str, need_s: float, fn, *a, collective: bool = True):
        if not self.fits(need_s, collective):
            self.skipped.append(name)
            if self.verbose:
                log(f"bench: section {name} skipped: needs ~{need_s:.0f} s, {self.left():.0f} s of the budget left")
            return self.marker(need_s)
        t0, prev = time.perf_counter(), self.current
        self.current = name
        if self.verbose:
            log(f"bench: [{self.used():.0f} s] section {name} (estimate {need_s:.0f} s)")
        try:
            return fn(*a)
        except BaseException:
            self.failed_in = self.failed_in or name  # the innermost section an error left
            raise
        finally:
            self.sections[name] = round(time.perf_counter() - t0, 2)
            if self.verbose:
                log(f"bench: [{self.used():.0f} s] section {name} done in {self.sections[name]:.1f} s")
            self.current = prev

    def heartbeat(self, every_s: float = 30.0) -> None:
        """A progress line on stderr every `every_s` while the run lasts: a long quiet section (the
        reference's CPU runs, a 137 GB host matrix) must not look like a hung command to a
        supervisor that watches the output."""
        def beat():
            while True:
                time.sleep(every_s)
                log(f"bench: [{self.used():.0f} s] running: {self.current or 'between sections'}")

        threading.Thread(target=beat, name="bench-heartbeat", daemon=True).start()

    def record(self) -> dict:
        return {"limit_s": self.limit_s, "reserve_s": self.reserve_s, "used_s": round(self.used(), 1),
                "skipped": list(self.skipped)}


class Report:
    """Rank 0's JSON line under construction. Sections store their results as they finish;
    `write()` prints the line once — at the end, or from the signal watcher when a time limit
    terminates the run (`truncated`: the line as far as it got). The watcher is a thread woken
    through signal.set_wakeup_fd, so the line goes out even while the main thread is blocked in a
    GPU or C call that would delay a Python-level handler; it then ends the process with
    os._exit (never an exec)."""

    def __init__(self, stream, budget: Budget | None = None):
        self.stream = stream
        self.budget = budget
        self.lock = threading.Lock()
        self.out: dict = {}
        self.written = False

    def __setitem__(self, key, value):
        with self.lock:
            self.out[key] = value

    def __getitem__(self, key):
        with self.lock:
            return self.out[key]

    def update(self, d: dict) -> None:
        with self.lock:
            self.out.update(d)

    def append(self, key, value) -> None:
        with self.lock:
            self.out.setdefault(key, []).append(value)

    def snapshot(self, **extra) -> dict:
        with self.lock:
            line = copy.deepcopy(self.out)
        if self.budget is not None:
            line["sections_s"] = dict(self.budget.sections)
            line["budget"] = self.budget.record()
        line["failures"] = list(FAILURES) or None
        line["warnings"] = list(WARNINGS) or None
        line.update(extra)
        return line

    def write(self, **extra) -> bool:
        line = self.snapshot(**extra)
        with self.lock:
            if self.written:
                return False
            self.written = True
            self.stream.write(json.dumps(line) + "\n")
            self.stream.flush()
        return True

    def on_uncaught(self) -> None:
        """An exception that ends the run (at N > 1 a section's error is fatal, every rank
        must stop) still leaves the line so far, marked truncated, with the error."""
        prev = sys.excepthook

        def hook(tp, value, tb):
            where = (self.budget.failed_in or self.budget.current) if self.budget is not None else None
            self.write(truncated=True, truncated_by="error", truncated_in=where,
                       error=f"{tp.__name__}: {str(value)[:300]}")
            prev(tp, value, tb)

        sys.excepthook = hook

    def watch_signals(self, exit_fn=None) -> None:
        """SIGTERM / SIGINT: write the line so far (truncated) and exit 128 + signal."""
        exit_fn = exit_fn or os._exit
        rfd, wfd = os.pipe()
        os.set_blocking(wfd, False)
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: None)  # installs CPython's C handler; the watcher acts
        signal.set_wakeup_fd(wfd, warn_on_full_buffer=False)

        def watcher():
            while True:
                b = os.read(rfd, 1)
                if not b:
                    return
                if b[0] not in (signal.SIGTERM, signal.SIGINT):
                    continue
                name = signal.Signals(b[0]).name
                where = self.budget.current if self.budget is not None else None
                log(f"bench: {name} during {where or 'the run'}: writing the line so far")
                self.write(truncated=True, truncated_by=name, truncated_in=where)
                stop_children()
                exit_fn(128 + b[0])
                return

        threading.Thread(target=watcher, name="bench-signal-watcher", daemon=True).start()


def expect(cond, msg) -> bool:
    """One of the bench's correctness checks (y against the oracle, the reference's own rows, the
    tree form, ...). A failure is logged and kept for the JSON line's `failures` and the run goes
    on to its end (at N > 1 every rank must still reach the same collectives), then exits 1."""
    if not cond:
        log(f"bench: CHECK FAILED: {msg}")
        FAILURES.append(str(msg)[:300])
    return bool(cond)


def kernel_family(variant: str) -> str:
    """The kernel template a dispatch variant name instantiates (the PMC summaries' key); the
    evenly placed multi-wave hop forms (hop8e_*) are a family of their own, so they never take
    counters recorded on the one-wave form."""
    for prefix, fam in (("rowlines", "gemv_rowblock_lines"), ("rowblk", "gemv_rowblock"), ("vec", "gemv_vec"),
                        ("scl", "gemv_scalar"), ("hopxl", "gemv_seq_hop_xl"), ("hop8e", "gemv_seq_hop_n8"),
                        ("hop", "gemv_seq_hop"),
                        ("seqx", "gemv_seq_x"), ("seq_", "gemv_seq"), ("panel", "gemv_seq_hop_panel")):
        if variant.startswith(prefix):
            return fam + ("_split" if variant.endswith("_splitk") else "")
    return variant


def pmc_summary(M: int, K: int, variant: str):
    """The newest committed rocprofv3 PMC summary (tools/pmc_traffic.py ->
    profiles/<round>/pmc_<family>_<M>x<K>.json) for this kernel family on an M x K shard: HBM bytes
    per launch (`traffic`), VALU busy, L2 hit rate, memory-side read latency and reads in flight,
    or None when no summary matches."""
    fam = kernel_family(variant)
    out, sources = {}, []
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "pmc_*.json"), recursive=True), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("kernel_family") == fam and d.get("M") == M and d.get("K") == K:
            # the newest summary first; a field it lacks (a counter pass it did not run) from the
            # next newest that has it
            got = {k: (float(f"{d[k]:.5g}") if isinstance(d[k], float) else d[k]) for k in (
                "hbm_bytes_per_launch", "traffic_over_algorithmic", "valu_busy", "l2_hit", "ea_read_latency_cyc",
                "ea_reads_in_flight", "dram_read_frac", "utcl1_miss_rate") if d.get(k) is not None and k not in out}
            if got:
                out.update(got)
                sources.append(os.path.relpath(path, REPO))
    if not out:
        return None
    out["source"] = sources[0] if len(sources) == 1 else sources
    return out


def launcher_cmd(argv: list[str], n: int, port: int) -> list[str]:
    """The driver's N-GPU command for this same invocation: torch.distributed.run with one rank
    per GPU on this node, rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def relay(cmd: list[str], env: dict | None = None) -> int:
    """Run `cmd` as a child process (never exec: the parent has not touched the GPU, and must not
    be replaced after it has), pass its stderr through, print the one JSON line its rank 0 wrote
    on stdout (every other stdout line goes to stderr), and return its exit code (1 if it exited
    0 without a JSON line)."""
    import subprocess

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    got: dict = {"line": None}

    def read():  # a thread, so a signal handler never re-enters the pipe's reader
        for ln in p.stdout:
            s = ln.strip()
            if s.startswith("{") and '"metric"' in s:
                got["line"] = s
            elif s:
                print(s, file=sys.stderr, flush=True)

    reader = threading.Thread(target=read, daemon=True)
    reader.start()

    def forward(signum, _frame):
        # a time limit on this process reaches the ranks too; rank 0 then writes its line so far
        # (truncated), which is passed on before this process exits
        p.send_signal(signum)
        try:
            p.wait(timeout=40)
        except subprocess.TimeoutExpired:
            p.kill()
        reader.join(timeout=10)
        if got["line"] is not None:
            print(got["line"], flush=True)
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    while p.poll() is None:  # never blocked inside Popen.wait, whose lock forward() needs
        time.sleep(0.1)
    rc = p.returncode
    reader.join()
    if got["line"] is not None:
        print(got["line"], flush=True)
    if rc == 0 and got["line"] is None:
        log("bench: the ranks exited without a JSON line")
        return 1
    return rc


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` with no launcher: start the N ranks ourselves (the reference's
        # own sweep is `mpiexec -n $np`, test.sh:5-11) and relay rank 0's line and the exit code
        sys.exit(relay(launcher_cmd(sys.argv[1:], args.gpus, free_port())))
    # stdout carries exactly one JSON line (rank 0): anything the runtimes print on fd 1
    # (RCCL's init banner, HIP messages) is sent to stderr instead.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = args.gpus
    budget = Budget(args.budget_s, verbose=rank == 0, reserve_s=10.0)
    report = Report(json_out, budget)
    if rank == 0:
        # from here on a time limit still gets a line: the fields known so far, "truncated": true
        report.update({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": n, "steps": args.steps,
                       "warmup": args.warmup, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                       "dtype": "f64",
                       "data": "synthetic (splitmix64 k/10000 values, bit-identical to the reference's %.4f text "
                               "inputs)"})
        report.watch_signals()
        report.on_uncaught()
        budget.heartbeat()
    # one process per GPU: CUDA-tensor / RCCL IPC between processes needs the dmabuf IPC mode on
    # this ROCm (the legacy handle path fails with hipIpcGetMemHandle: invalid argument); set before
    # the HIP runtime starts. With N > 1, RCCL logs at INFO to a per-rank file that rccl_report()
    # reads back (the transport of every connection: P2P/IPC over xGMI, or SHM / NET); the WARN and
    # ERROR lines of that file are passed on to stderr, so a caller's NCCL_DEBUG=WARN (or any
    # level up to INFO; the pool's boxes export VERSION) loses nothing. A caller who sends RCCL's
    # log to a file of their own (NCCL_DEBUG_FILE) keeps it untouched, and the report is skipped.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rccl_log, caller_debug = None, os.environ.get("NCCL_DEBUG")
    caller_nccl = {k: os.environ.get(k) for k in ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE")}
    if world > 1 and "NCCL_DEBUG_FILE" not in os.environ:
        rccl_log = f"/tmp/mvg_rccl_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('RANK', '0')}.log"
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P", NCCL_DEBUG_FILE=rccl_log)
    import torch
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd import multiplier as mm

    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch N > 1 with torch.distributed.run")
    # MVG_SAME_DEVICE=1 (rehearsal on a one-GPU machine): every rank on GPU 0; RCCL refuses two
    # ranks on one device of one host, so each rank names its own host and the ranks talk over
    # loopback sockets (timings then mean nothing; the N > 1 code path runs end to end)
    if os.environ.get("MVG_SAME_DEVICE") == "1" and world > 1:
        os.environ.setdefault("NCCL_HOSTID", f"mvg-rank-{rank}")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        local = 0
    torch.cuda.set_device(local)
    # MVG_BENCH_FORCE_DIST=1 runs the one-process-per-GPU path (process group, RCCL comm from the
    # group, shared-memory distribution, root sends) even at world size 1, to rehearse it on a
    # one-GPU box
    distributed = world > 1 or os.environ.get("MVG_BENCH_FORCE_DIST") == "1"
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    budget.distributed, budget.device = distributed, f"cuda:{local}"
    if args.event_every is None:
        args.event_every = 5 if distributed else -1

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    budget.current = "headline"
    t_head = time.perf_counter()
    R = args.rows if args.rows is not None else SHARD * n
    C = args.cols
    comm = mm.Comm.from_process_group(local) if distributed else mm.Comm.init_all([local])
    eng = mm.Multiplier(args.alg, R, C, comm)
    sh = eng.shard(0)
    eng.fill_synth()
    eng.sync()

    # settle: the first second or so of a fresh box runs the kernel slow (its shader clock leaving
    # idle; on a box just handed over, 310 us for ~1 s, then 296 — profiles/r05/fresh_box), and
    # W = 5 warm-up steps (1.5 ms) do not cover it (round 5: the headline at 311.5 us while the
    # same shape ran 297 us later in the same process, profiles/r05/r5r). So untimed multiplies
    # run in bursts for at least --settle-s (1.5 s: the slow phase is steady in itself, so only
    # time outlasts it; under continuous load it lasted 0.5-0.75 s, profiles/r05/settle/) and until
    # the per-step time is steady, at most --settle-max-s (settle()), then the W warm-up steps; the
    # line records it as `settle`, with a sample of the step time every 0.25 s.
    # From the settle to the end of the timed steps the GPU never idles for more than a
    # synchronize: an idle gap of >= 10 ms before 20 launches (a sleep, or the 36 ms of a
    # gc.collect()) slows them by 0.6-1.2 % as the shader clock dips (profiles/r05/idle_gap/), so
    # the collection runs before the settle and the collector stays off until the timed steps end.
    gc.collect()
    gc.disable()
    try:
        vram_wait = wait_vram_cleared(local)  # VRAM a previous process freed may still be being cleared
        settled = (settle(eng, args.settle_s, args.settle_max_s, distributed, local)
                   if args.settle_s > 0 else None)
        # the W warm-up steps already run with kernel timing on, so the timing events' first use
        # (their creation, the runtime's first timestamped marker) falls outside the timed region
        eng.kernel_timing(args.event_every)
        for _ in range(args.warmup):
            eng.multiply()
        eng.kernel_timing(args.event_every)  # waits for the warm-up, resets the counts: only the K timed steps
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.multiply()
        eng.sync()
        barrier()
        elapsed = time.perf_counter() - t0
    finally:
        gc.enable()
    kt = eng.kernel_ms()
    eng.kernel_timing(0)

    kernel_by_rank = per_rank(kt.avg_ms, distributed, local)
    t = torch.tensor([elapsed, kt.avg_ms], dtype=torch.float64, device=f"cuda:{local}")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms = float(t[0]), float(t[1])

    # algorithmic bytes: every GPU reads its A shard once, its x segment once, writes its y piece
    def shard_bytes(s):
        part = R if args.alg == "colwise" else s.y_len
        return 8 * (s.n_rows * s.n_cols + s.n_cols + part)

    per_gpu = shard_bytes(sh)
    total_bytes = sum(shard_bytes(mm.plan_shard(args.alg, R, C, n, r)) for r in range(n))
    value = total_bytes * args.steps / elapsed / 1e9
    achieved = per_gpu / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None

    # y of the timed steps, on rank 0: every element must lie in [0, C * 0.9999^2] (inputs are in
    # [0, 0.9999]); exact parity is checked against the reference restatement in cpu_baseline
    # (N = 1) and by tests/.
    y = eng.collect()
    if rank == 0:
        expect(np.all(np.isfinite(y)) and y.min() >= 0.0 and y.max() <= C * 0.9999 ** 2, "y out of range")
        pmc = pmc_summary(sh.n_rows, sh.n_cols, kernel_name(sh)) or {}
        report.update({
            "settle": settled,
            "vram_wait": vram_wait,
            "value": round(value, 1),
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "gflops": round(2 * R * C * args.steps / elapsed / 1e9, 1),  # whole job, 2 flops per element of A
            "config": {
                "workload": ("config 2 weak-scaled: " if (args.rows, args.cols) == (None, SHARD) else "")
                            + f"{args.alg} of a ({R} x {C}) fp64 matrix, "
                            f"{sh.n_rows} x {sh.n_cols} shard per GPU, device-resident",
                "alg": args.alg, "R": R, "C": C, "shard": [sh.n_rows, sh.n_cols],
                "parallelism": f"{args.alg} over {n} GPU(s), exchange "
                               + {"rowwise": "ncclGather", "colwise": "ncclReduce", "blockwise": "row ncclReduce + leader ncclGather"}[args.alg],
                "bytes_per_step": total_bytes,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "valu_busy": pmc.get("valu_busy"),
                "l2_hit": pmc.get("l2_hit"),
                "kernel": kernel_name(sh) + ", per GPU",
                "kernel_ms": round(kernel_ms, 5),
                "kernel_timing": timing_note(args.event_every, args.steps),
                "kernel_ms_by_rank": kernel_by_rank,
                "bytes_per_launch": per_gpu,
                "pmc": pmc or None,
            },
        })
    budget.sections["setup_and_headline"] = round(time.perf_counter() - T_START, 2)
    budget.sections["headline"] = round(time.perf_counter() - t_head, 2)
    budget.current = None

    # ---- the sections after the headline, each within the budget (Budget.run). Their parity
    # checks never raise (expect(): recorded, exit code 1 at the end). Any other error — the
    # environment's: out of memory, a missing reference binary — is recorded in the section's
    # place in one process (no other rank waiting in a collective) and ends the run with N > 1
    # ranks, as it must.
    def guarded(fn, *a):
        if distributed:
            return fn(*a)
        try:
            return fn(*a)
        except Exception as exc:
            import traceback

            traceback.print_exc()
            WARNINGS.append(f"{getattr(fn, '__name__', fn)}: {type(exc).__name__}: {str(exc)[:200]}")
            return {"failed": f"{type(exc).__name__}: {str(exc)[:300]}"}

    def section(name, need_s, fn, *a, collective=True):
        return budget.run(name, need_s, guarded, fn, *a, collective=collective)

    # the same workload in bit-exact mode (the reference's sequential sums, bit for bit)
    y_exact = None
    if not args.no_exact:
        got = section("exact", est_exact(per_gpu, args.steps), exact_section, args, eng, n, rank, local,
                      distributed, barrier, per_gpu, total_bytes, y)
        exact, y_exact = got if isinstance(got, tuple) else (got, None)
        if rank == 0:
            report["exact"] = exact

    # CPU baseline: rank 0 at N = 1 only (the reference's own executable beside its port)
    if rank == 0 and n == 1 and not args.no_cpu_baseline:
        big = big_sample_rows(args, args.alg, R, C)
        cpu = section("cpu_baseline", est_cpu_baseline(args, R, C, big_rows=big), cpu_baseline, args, args.alg, R, C,
                      y, y_exact, None, None, None, ("spread", "compact"),
                      tuple(int(p) for p in args.cpu_sweep.split(",") if p.strip()), big, collective=False)
        same_port = cpu.pop("exact_vs_port", None) if isinstance(cpu, dict) else None
        same_ref = cpu.pop("exact_vs_reference", None) if isinstance(cpu, dict) else None
        report["cpu_baseline"] = cpu
        with report.lock:
            ex = report.out.get("exact")
            if isinstance(ex, dict) and "value" in ex:
                # rowwise: the exact y against the oracle port's y (full matrix) and against the
                # real reference's own y (its sample rows), bit for bit
                ex["bit_identical_to_port"] = same_port
                ex["bit_identical_to_reference_sample"] = same_ref

    # BASELINE configs 3-5 at their own sizes on these N GPUs, and the end-to-end loops (the
    # headline's and the configs'), in three passes (config_passes): every config's
    # device-resident steps first, then the end-to-end loops smallest A first, then (N = 1) the
    # configs' CPU baselines. The main engine's HBM is released first (config 4 is 128 GiB per
    # GPU at N = 1); the headline's end-to-end loop runs on a fresh engine of its own.
    eng.destroy()
    if rank == 0 and not args.no_configs:
        report["configs"] = []

    def headline_e2e():
        def run():
            e = mm.Multiplier(args.alg, R, C, comm)
            try:
                return end_to_end(args, e, mm, R, C, rank, distributed, barrier, y, total_bytes, local, budget)
            finally:
                e.destroy()

        return section("end_to_end", est_e2e(total_bytes, n, args.e2e_iters, distributed), run)

    config_passes(
        args, n, rank, budget, report,
        run_device=lambda k: config_device(args, mm, comm, n, rank, local, distributed, barrier, budget, guarded, k),
        run_e2e=lambda k, yk: config_e2e(args, mm, comm, n, rank, local, distributed, barrier, budget, guarded, k, yk),
        run_cpu=lambda k, yk: config_cpu(args, budget, guarded, k, yk),
        headline_e2e=headline_e2e, headline_bytes=8 * R * C)

    # several x per pass over A, rank 0 at N = 1
    if rank == 0 and n == 1 and not args.no_multi:
        report["multi_vector"] = section("multi_vector", 8.0, multi_vector_section, local, collective=False)

    # the text loader on config 2's input file, rank 0 at N = 1
    if rank == 0 and n == 1 and not args.no_loader:
        report["loader"] = section("loader", est_loader(R, C), loader_section, R, C, collective=False)

    budget.current = "teardown"
    rccl = rccl_report(rccl_log, distributed, rank) if distributed else None
    if rccl is not None:
        rccl["caller_NCCL_DEBUG"] = caller_debug
    if rank == 0:
        from matvec_mpi_multiplier_amd._lib import runtime_info

        # the RCCL and HIP runtime the rank sections ran on (PyTorch's bundled copies when the
        # package imported torch first, _lib._torch_first); the single-process child reports its own
        rt = runtime_info()
        rt["executables"] = executable_runtime(args.alg)  # bin/multiplier_*: /opt/rocm's, not PyTorch's
        report["runtime"] = rt
        if rccl is not None:
            rccl["version"], rccl["path"] = rt.get("rccl_version"), rt.get("rccl_path")
        report["rccl"] = rccl
        if args.alg == "rowwise" and C == SHARD and R >= SHARD:
            # the weak-scaled matrix's first 16384 rows are config 2's matrix (global index i*C + j),
            # and a row's sum does not depend on P: config 2's reference rows check every N
            report["reference_rows"] = reference_rows_check("config 2", "rowwise", R, C, n, y, y_exact)

    comm.destroy()
    if distributed:
        dist.destroy_process_group()
    budget.current = None
    if rank == 0:
        if n > 1:
            # the executables' one-process-drives-N-GPUs path (ncclCommInitAll, grouped exchange),
            # which the rank-per-GPU sections above never run; the other ranks have exited
            if single_process_blocker(n):  # nothing to run here: record why, whatever the budget
                sp = single_process_section(args, n, R, C, caller_nccl, None, budget)
            else:
                sp = budget.run("single_process", est_single_process(R, C, n), single_process_section, args, n, R,
                                C, caller_nccl, None, budget, collective=False)
            report["single_process"] = sp
            if isinstance(sp, dict) and sp.get("error"):
                WARNINGS.append(f"single_process: the MVG_NGPUS={n} executable failed (rc {sp.get('rc')}): "
                                f"{sp['error'][-200:]}")
        else:
            report["single_process"] = None
        report.write()
    if FAILURES:
        sys.exit(1)


# ---- section time estimates (s) for the budget: generous upper bounds from the round-4/5 box
# records (sections_s of profiles/r05 bench lines); a section runs only if its estimate fits
GEN_GBPS = 20.0    # host synthetic fill + first touch (16 threads; r05: 137 GB filled, pinned and
PIN_GBPS = 40.0    #   distributed 3 times in 10 s) / hipHostRegister of a host matrix
H2D_GBPS = 40.0    # per-GPU host -> device distribution (56 measured: 0.7 of it)
REF_TEXT_GBPS = 0.08  # the reference's fscanf load of its text input, per byte of A (with the file write)


def est_exact(per_gpu, steps):
    return 4.0 + 3 * per_gpu / 6e12 * (2 * steps + 100)


SHM_SETUP_GBPS = 3.0  # N > 1: the /dev/shm matrix (4 KiB tmpfs pages: shmem huge pages are off on the
                      # boxes, no hugetlb pool) filled by the ranks, each with its share of the CPU
                      # quota, then page-locked. Round 6 probes, 32 GiB: 3.4-6.8 GB/s for the whole
                      # node at 1, 4 or 8 processes (the tmpfs page allocation, not the CPUs: first
                      # touch, MADV_POPULATE_WRITE or pinning first all land there), against 1.45
                      # GB/s when each of 4 ranks ran the whole quota's threads (round 5's 0.8 GB/s)
                      # and 57-63 GB/s for the N = 1 anonymous (THP) matrix (profiles/r06/host_setup*)


def est_e2e(total_bytes, n, iters, distributed):
    if distributed:
        gen, pin = total_bytes / (SHM_SETUP_GBPS * 1e9), 0.0
    else:
        gen, pin = total_bytes / (GEN_GBPS * 1e9), total_bytes / (PIN_GBPS * 1e9)
    per_iter = total_bytes / n / (H2D_GBPS * 1e9) + 0.05
    root_send = iters * total_bytes / (H2D_GBPS * 1e9) if distributed else 0.0
    return 4.0 + gen + pin + iters * per_iter + root_send


def est_config(per_gpu, steps):
    # engine create (memset + warm-up), fill, warm-up, tree + exact steps, y copies
    return 6.0 + per_gpu / 2e10 + 2 * per_gpu / 6e12 * (steps + 40)


def est_ref_run(nbytes, P):
    # one run of the reference's executable on an nbytes sample: its text input written and read
    # (fscanf), then its 100-iteration loop (~2.9 GB/s at P = 1, ~4-5 at P = 16 on the EPYC box)
    rate = 2.5e9 if P == 1 else 3.5e9
    return 3.0 + nbytes / (REF_TEXT_GBPS * 1e9) / 10 + 100 * nbytes / rate


def est_cpu_baseline(args, R, C, ref_rows=None, big_rows=None, sweep=True, port_bytes=None, cpu_seconds=None,
                     placements=2):
    port_bytes = min(8 * R * C, args.cpu_sample_bytes if port_bytes is None else port_bytes)
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    # inputs generated, the first timed iteration, then about cpu_seconds of iterations
    t = 3.0 + port_bytes / (6e9) + port_bytes / 4e9 + 2 * cpu_seconds
    small = 8 * min(R, ref_rows or args.ref_rows) * C
    t += placements * est_ref_run(small, 16)
    if sweep:
        t += sum(est_ref_run(small, p) for p in (1, 2, 4, 8))
    if big_rows:
        big = 8 * min(R, big_rows) * C
        t += est_ref_run(big, 16) + est_ref_run(big, 1)
    return t


def est_loader(R, C):
    return 5.0 + 7 * R * C / 0.8e9 + 2 * 8 * R * C / (GEN_GBPS * 1e9)


def est_single_process(R, C, n):
    return 30.0 + 60 * 8 * R * C / n / 7e12 + 8 * R * C / 20e9


def settle(e, min_s, max_s, distributed, local, burst=20, tol=0.01):
    """Untimed multiplies in bursts of `burst`, each timed by the wall clock between device syncs,
    until the last three bursts' per-step times agree within `tol` and at least `min_s` has
    passed, or `max_s` has (at N > 1 every rank runs bursts until every rank is done: the decision
    is all-reduced, each multiply being a collective). Returns what it did: seconds, bursts, and
    the first and last bursts' time per step, and a sample every 0.25 s."""
    t0, per, trace, next_mark = time.perf_counter(), [], [], 0.0
    while True:
        tb = time.perf_counter()
        for _ in range(burst):
            e.multiply()
        e.sync()
        per.append((time.perf_counter() - tb) / burst)
        el = time.perf_counter() - t0
        if el >= next_mark:  # a sample every 0.25 s: how long a slow phase lasted
            trace.append([round(el, 2), round(per[-1] * 1e6, 1)])
            next_mark += 0.25
        last = per[-3:]
        steady = len(last) == 3 and max(last) - min(last) <= tol * min(last)
        done = el >= max_s or (el >= min_s and steady)
        if distributed:
            import torch
            import torch.distributed as dist

            t = torch.tensor([1.0 if done else 0.0], dtype=torch.float64, device=f"cuda:{local}")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            done = float(t[0]) >= 1.0
        if done:
            return {"s": round(el, 2), "bursts": len(per), "steady": steady,
                    "first_us_per_step": round(per[0] * 1e6, 1), "last_us_per_step": round(per[-1] * 1e6, 1),
                    "trace_s_us": trace}


def _sysfs_vram_used(local):
    """Bytes of GPU `local`'s VRAM its kernel driver counts as used (every process on the GPU),
    from the device's own sysfs node (its PCI address: the host's other GPUs are listed too);
    None when unreadable."""
    import torch

    try:
        p = torch.cuda.get_device_properties(local)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/mem_info_vram_used") as f:
            return int(f.read().strip())
    except Exception:  # no such device, no sysfs node, not a ROCm build: nothing to wait on
        return None


def vram_pending_bytes(local):
    """VRAM the driver still counts as used beyond what this process holds (hipMemGetInfo's
    total - free): memory an earlier section or process freed that the kernel driver is still
    clearing. It clears freed VRAM in the background, and while it does an HBM-bound kernel runs
    up to 5 % slow: config 2's GEMV at 301-309 us instead of 294 for 3.9 s after a 128 GiB
    hipFree, the sysfs count dropping back exactly when the kernel recovers
    (profiles/r06/vram_clear/). None when sysfs does not say."""
    import torch

    used = _sysfs_vram_used(local)
    if used is None:
        return None
    free, total = torch.cuda.mem_get_info(local)
    return max(0, used - (total - free))


_VRAM_OFFSET = {}  # per GPU: bytes sysfs counts that never clear (learned after one timeout)


def wait_vram_cleared(local, timeout_s=10.0, slack=1 << 30, poll_s=0.05):
    """Before a timed section: wait (untimed, at most `timeout_s`) until the driver has cleared
    the VRAM freed before it — by the previous config's engine, or by the previous process on
    the GPU — so the section is not timed while the driver's clearing shares HBM with it (137 GB
    clear in about 4 s). What it found and how long it waited goes into the line. A count that
    has not moved at all by the time limit is not clearing but something sysfs counts and this
    process's view does not: it becomes that GPU's offset, and later waits do not wait on it. Not
    at MVG_SAME_DEVICE=1 (every rank's memory is on one GPU there, so this process's view never
    accounts for it all)."""
    if os.environ.get("MVG_SAME_DEVICE") == "1":
        return None
    t0 = time.perf_counter()
    raw = vram_pending_bytes(local)
    if raw is None:
        return None
    off = _VRAM_OFFSET.get(local, 0)
    first = pend = max(0, raw - off)
    while pend > slack and time.perf_counter() - t0 < timeout_s:
        time.sleep(poll_s)
        pend = max(0, vram_pending_bytes(local) - off)
    out = {"pending_gib": round(first / 2 ** 30, 2), "waited_s": round(time.perf_counter() - t0, 2),
           "left_gib": round(pend / 2 ** 30, 2)}
    if pend > slack and abs(pend - first) <= slack:
        _VRAM_OFFSET[local] = off + pend
        out["offset_learned_gib"] = round((off + pend) / 2 ** 30, 2)
    return out


def wait_devices_cleared(n, local, timeout_s=10.0, slack=1 << 30, poll_s=0.05):
    """wait_vram_cleared over GPUs 0 .. n-1 before the single-process child takes all of them:
    the rank processes have just exited, and the driver clears what they held. Only this
    process's own GPU holds anything of ours; on the others every counted byte is pending."""
    if os.environ.get("MVG_SAME_DEVICE") == "1":
        return None
    t0 = time.perf_counter()

    def pending():
        tot = 0
        for d in range(n):
            v = vram_pending_bytes(d) if d == local else _sysfs_vram_used(d)
            if v is None:
                return None
            tot += v
        return tot

    first = pend = pending()
    if first is None:
        return None
    while pend > n * slack and time.perf_counter() - t0 < timeout_s:
        time.sleep(poll_s)
        pend = pending()
    return {"pending_gib": round(first / 2 ** 30, 2), "waited_s": round(time.perf_counter() - t0, 2),
            "left_gib": round(pend / 2 ** 30, 2)}


def warm(e, min_launches, distributed, local, seconds=0.3):
    """Untimed multiplies before a supplementary timed section: at least `min_launches`, and about
    `seconds` of them, so that the section is timed in a steady state rather than right after the
    host work between sections (y checks, D2H copies) has idled the GPU: the launches after such a
    gap run slow (round 4 traces: the tree kernel's first launch after a 16 ms gap 322 us, then
    300; round 5: 20 launches after a 10-200 ms gap 0.6-1.2 % slower, and 0.3 s of load before
    them undoes it, profiles/r05/idle_gap/). Every rank runs the same count (each multiply has a
    collective at N > 1)."""
    import torch
    import torch.distributed as dist

    t0 = time.perf_counter()
    for _ in range(min_launches):
        e.multiply()
    e.sync()
    per = (time.perf_counter() - t0) / max(1, min_launches)
    more = int(min(2000, max(0.0, seconds / max(per, 1e-6) - min_launches)))
    if distributed:
        t = torch.tensor([float(more)], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        more = int(t[0])
    for _ in range(more):
        e.multiply()
    e.sync()


def single_process_blocker(n):
    """Why this box cannot run the one-process-drives-N-GPUs form (None when it can)."""
    import torch

    have = torch.cuda.device_count()
    if have < n or os.environ.get("MVG_SAME_DEVICE") == "1":
        return (f"needs {n} devices in one process, {have} visible"
                + (" (MVG_SAME_DEVICE rehearsal: every rank on one GPU)" if os.environ.get("MVG_SAME_DEVICE") == "1" else ""))
    return None


def single_process_section(args, n, R, C, caller_nccl=None, exe=None, budget=None):
    """The drop-in executables' single-process form of the same workload: ONE process drives all
    N GPUs (mvg_comm_init_all -> ncclCommInitAll over N devices, the grouped ncclCommSplit and the
    exchange grouped over the local devices, csrc/engine.cpp), which the one-rank-per-GPU
    sections above never run. Rank 0 starts `MVG_NGPUS=N MVG_SYNTH=device bin/multiplier_<alg>
    R C` as a child process once the process group is gone, and records its device-resident line
    and its y against config 2's reference rows. A failure is recorded here, never fatal; the
    reference's own grid and gather: multiplier_blockwise.c:299-306, :144-210. The child's time
    limit is what is left of the budget (at most 300 s); a failed run is also a top-level
    warning of the line (main)."""
    import re
    import shutil
    import tempfile

    why = single_process_blocker(n)
    if why:
        return {"ran": False, "why": why}
    exe = exe or os.path.join(REPO, "bin", f"multiplier_{args.alg}")
    if not os.access(exe, os.X_OK):
        return {"ran": False, "why": f"{os.path.relpath(exe, REPO)} not built"}
    work = tempfile.mkdtemp(prefix="mvg_single_")
    try:
        ypath = os.path.join(work, "y.txt")
        drop = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT"}
        env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC")}
        for k, v in (caller_nccl or {}).items():  # RCCL's logging as the caller set it, not ours
            env.pop(k, None)
            if v is not None:
                env[k] = v
        iters = 50
        env.update(MVG_NGPUS=str(n), MVG_SYNTH="device", MVG_ITERS=str(iters), MVG_Y_OUT=ypath)
        cmd = [exe, str(R), str(C)]
        cleared = wait_devices_cleared(n, int(os.environ.get("LOCAL_RANK", "0")))
        t0 = time.perf_counter()
        limit = 300.0 if budget is None else max(10.0, min(300.0, budget.left() - 5.0))
        r = run_child(cmd, limit, cwd=work, env=env)
        wall = time.perf_counter() - t0
        out = {"ran": True, "command": f"MVG_NGPUS={n} MVG_SYNTH=device MVG_ITERS={iters} "
                                      f"bin/multiplier_{args.alg} {R} {C}", "rc": r.returncode,
               "wall_s": round(wall, 2), "vram_wait": cleared}
        m = re.search(r"device-resident: ([\d.]+) ms per multiply, ([\d.]+) GB/s aggregate; GEMV kernel ([\d.]+) ms",
                      r.stdout)
        if r.returncode != 0 or not m or not os.path.exists(ypath):
            # recorded, not counted as a failed check: the rank sections' scaling line stands
            # (a wrong y from a run that did finish is counted, below)
            out["error"] = (r.stdout[-300:] + " | " + r.stderr[-500:]).strip()
            return out
        out.update(ms_per_step=float(m.group(1)), value=float(m.group(2)), unit="GB/s",
                   kernel_ms=float(m.group(3)))
        m2 = re.search(r"end-to-end \(([^)]*)\): mean ([\d.]+) s", r.stdout)
        if m2:
            out["end_to_end_s"] = float(m2.group(2))
        out["runtime"] = parse_runtime_line(r.stdout)
        y = np.loadtxt(ypath, dtype=np.float64, ndmin=1)
        expect(y.shape == (R,), f"single-process y has {y.shape} elements, want {R}")
        if args.alg == "rowwise" and C == SHARD and R >= SHARD and y.shape == (R,):
            out["reference_rows"] = reference_rows_check("config 2", args.alg, R, C, n, y, None)
        return out
    except Exception as exc:  # recorded, never fatal: the rank sections' line still prints
        return {"ran": False, "error": f"{type(exc).__name__}: {str(exc)[:300]}"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def timing_note(every, steps):
    """How `kernel_ms` was measured (mvg_engine_kernel_timing): one event pair spanning the timed
    GEMVs, or events bracketing every Nth one."""
    if every == -1:
        return (f"span: one HIP event pair from the first timed GEMV's start to the stream's end at the closing "
                f"sync, / {steps} launches (no marker between the launches; a span holding any other write to "
                f"the shard is dropped)")
    return f"events bracketing every {every}th GEMV on the engine stream, mean over the bracketed launches"


def executable_runtime(alg):
    """The RCCL and HIP runtime the drop-in executables bind (MVG_RUNTIME_ONLY=1
    bin/multiplier_<alg>: the `runtime:` line, no device work), for the line's `runtime` beside
    the rank sections' own; None when the executable is missing or says nothing."""
    exe = os.path.join(REPO, "bin", f"multiplier_{alg}")
    if not os.access(exe, os.X_OK):
        return None
    try:
        r = run_child([exe], 30, env={**os.environ, "MVG_RUNTIME_ONLY": "1"})
    except Exception:
        return None
    return parse_runtime_line(r.stdout)


def parse_runtime_line(text):
    """The executables' "runtime: RCCL <code> (<path>), HIP <version> (<path>)" line (the RCCL
    and HIP runtime that process ran on), as runtime_info() reports them; None without one."""
    import re

    from matvec_mpi_multiplier_amd._lib import rccl_version_text

    m = re.search(r"runtime: RCCL (\d+) \(([^)]*)\), HIP (\d+) \(([^)]*)\)", text or "")
    if not m:
        return None
    origin = (lambda p: "pytorch" if "/torch/lib/" in p else "rocm" if "/rocm" in p else "unknown")
    return {"rccl_version": rccl_version_text(int(m.group(1))), "rccl_version_code": int(m.group(1)),
            "rccl_path": m.group(2), "rccl_origin": origin(m.group(2)),
            "hip_runtime_version": int(m.group(3)), "hip_path": m.group(4), "hip_origin": origin(m.group(4))}


def exact_section(args, eng, n, rank, local, distributed, barrier, per_gpu, total_bytes, y_tree):
    """The same workload with the engine in bit-exact mode (mvg_engine_set_exact: every row the
    reference's own sequential chain of rounded products and adds, mvg_gemv_exact): step rate,
    the exact kernel's HBM fraction, and its y against the tree-summed y (<= 1e-12). Bit
    identity with the reference is checked against the oracle port's y in cpu_baseline."""
    import torch
    import torch.distributed as dist

    steps = max(10, args.steps // 2)

    def run_exact():
        warm(eng, max(2, args.warmup // 4), distributed, local)
        eng.kernel_timing(args.event_every)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.multiply()
        eng.sync()
        barrier()
        el = time.perf_counter() - t0
        kt = eng.kernel_ms()
        eng.kernel_timing(0)
        t = torch.tensor([el, kt.avg_ms], dtype=torch.float64, device=f"cuda:{local}")
        if distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kms = float(t[0]), float(t[1])
        return el, kms, eng.collect(), exact_kernel_name(eng)

    # 1) repeated multiplies of one distribution (the bench's step): from the second multiply on,
    #    the engine's column-panel copy of the shard (rebuilt once, during the warmup)
    eng.set_exact(True)
    try:
        el, kms, y, kernel = run_exact()
    finally:
        eng.set_exact(False)
    # 2) the row-major exact kernels, which every multiply of a fresh distribution runs (the
    #    drop-in executables: distribute + multiply each iteration, MVG_EXACT=1)
    had = os.environ.get("MVG_NO_PANELS")
    os.environ["MVG_NO_PANELS"] = "1"
    eng.set_exact(True)
    try:
        rel_, rkms, y_rm, rkernel = run_exact()
    finally:
        eng.set_exact(False)
        if had is None:
            del os.environ["MVG_NO_PANELS"]
        else:
            os.environ["MVG_NO_PANELS"] = had
    frac = (lambda ms: round(per_gpu / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if ms > 0 else None)
    out = {"semantics": "mvg_engine_set_exact: y bit-identical to the reference's sequential sums; "
                        "repeated multiplies of one distribution (device-resident), which run on the "
                        "engine's column-panel copy of the shard from the second multiply on (built "
                        "during the warmup, DESIGN.md §4b); `row_major`: the kernels a fresh "
                        "distribution runs (the executables' MVG_EXACT=1 loop)",
           "value": round(total_bytes * steps / el / 1e9, 1), "unit": "GB/s", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 4), "gflops": round(2 * eng.R * eng.C * steps / el / 1e9, 1),
           "kernel": kernel,
           "kernel_ms": round(kms, 5),
           "roofline_frac": frac(kms),
           "pmc": pmc_summary(eng.shard(0).n_rows, eng.shard(0).n_cols, kernel),
           "row_major": {"value": round(total_bytes * steps / rel_ / 1e9, 1), "ms_per_step": round(rel_ / steps * 1e3, 4),
                         "kernel": rkernel, "kernel_ms": round(rkms, 5), "roofline_frac": frac(rkms),
                         "pmc": pmc_summary(eng.shard(0).n_rows, eng.shard(0).n_cols, rkernel)}}
    if rank == 0:
        rel = float(np.max(np.abs(y - y_tree) / np.abs(y_tree)))
        expect(rel <= 1e-12, f"exact y differs from the tree-summed y by {rel}")
        expect(np.array_equal(y, y_rm), "the panel and row-major exact kernels differ")
        out["max_rel_vs_tree"] = rel
    return out, y


def multi_vector_section(local, M=SHARD, K=SHARD, launches=20):
    """mvg_gemv_multi (several x per pass over A; beyond the reference) on a
    config-2-sized A: for nv = 2, 4, 8, 16 the kernel's mean time (HIP events, `launches` back to
    back), the rate at which it reads A and its algorithmic bytes (A once, every x and y), and
    the speed-up over nv separate mvg_gemv calls timed the same way. Each vector's y is checked
    against the single-vector kernel's (<= 1e-12)."""
    import torch

    from matvec_mpi_multiplier_amd import multiplier as mm
    from matvec_mpi_multiplier_amd._lib import check, lib

    s = torch.cuda.current_stream(local).cuda_stream
    nvmax = 16
    dA, dX, dY, dy = mm.DeviceBuffer(M * K), mm.DeviceBuffer(K * nvmax), mm.DeviceBuffer(M * nvmax), mm.DeviceBuffer(M)
    try:
        check(lib.mvg_synth_fill_device(dA.ptr, K, M, K, 0, 0, K, 42, s), "fill A")
        for v in range(nvmax):  # vector v: seed 4242 + v
            check(lib.mvg_synth_fill_device(dX.ptr + 8 * K * v, K, 1, K, 0, 0, K, 4242 + v, s), "fill x")
        check(lib.mvg_stream_sync(s), "sync")
        cleared = wait_vram_cleared(local)  # the end-to-end engines before it freed up to 128 GiB

        def t(fn):
            fn()
            torch.cuda.synchronize(local)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(launches):
                fn()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / launches

        single = t(lambda: lib.mvg_gemv(dA.ptr, K, dX.ptr, dy.ptr, M, K, s))
        out = {"shape": [M, K], "single_ms": round(single, 5), "nv": {}, "vram_wait": cleared}
        worst = 0.0
        for nv in (2, 4, 8, 16):
            ms = t(lambda: lib.mvg_gemv_multi(dA.ptr, K, dX.ptr, K, dY.ptr, M, M, K, nv, s))
            Y = dY.download(M * nv).reshape(nv, M)
            for v in range(nv):
                check(lib.mvg_gemv(dA.ptr, K, dX.ptr + 8 * K * v, dy.ptr, M, K, s), "gemv")
                check(lib.mvg_stream_sync(s), "sync")
                y1 = dy.download()
                worst = max(worst, float(np.max(np.abs(Y[v] - y1) / np.abs(y1))))
            out["nv"][str(nv)] = {
                "kernel_ms": round(ms, 5),
                "A_GBps": round(8 * M * K / (ms * 1e-3) / 1e9, 1),
                "algorithmic_GBps": round(8 * (M * K + nv * (K + M)) / (ms * 1e-3) / 1e9, 1),
                "speedup_vs_separate": round(nv * single / ms, 3),
                "kernel": lib.mvg_gemv_multi_variant_name(lib.mvg_gemv_multi_auto_variant(K, K, M, K, nv)).decode(),
            }
        expect(worst <= 1e-12, f"multi-vector y differs from the single-vector y by {worst}")
        out["max_rel_vs_single"] = worst
        return out
    finally:
        for b in (dA, dX, dY, dy):
            b.free()


def host_threads():
    """The library's host thread count (csrc/host.cpp host_thread_count): $MVG_THREADS, else the
    process's CPUs capped by its cgroup quota, at most 64."""
    from matvec_mpi_multiplier_amd.hostshare import cpu_quota

    if os.environ.get("MVG_THREADS"):
        return max(1, min(64, int(os.environ["MVG_THREADS"])))
    return cpu_quota()


def loader_section(R, C):
    """The reference's input file for this workload (./data/matrix_R_C.txt, "%.4f" tokens,
    matr_utils.c:42-62), written to a scratch directory and read back by mvg_load_matr (mmap +
    threads, bit-identical to fscanf "%lf"): its parse rate on this host, and the matrix it gives
    against the synthetic generator's, bit for bit. The file is removed afterwards."""
    import shutil
    import tempfile

    from matvec_mpi_multiplier_amd import multiplier as mm

    work = tempfile.mkdtemp(prefix="mvg_loader_")
    try:
        path = os.path.join(work, mm.build_matrix_filename(R, C))
        t0 = time.perf_counter()
        mm.write_matr_synth(path, R, C, 42)
        wrote = time.perf_counter() - t0
        nbytes = os.path.getsize(path)
        best = None
        for _ in range(2):  # the first pass also pages the file in
            t0 = time.perf_counter()
            A = mm.load_matr(R, C, work)
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        same = bool(np.array_equal(A, mm.synth_host(R, C, 42)))
        expect(same, "the loader's matrix differs from the synthetic values its file holds")
        del A
        return {"file": os.path.basename(path), "text_bytes": nbytes, "parse_s": round(best, 4),
                "GBps_text": round(nbytes / best / 1e9, 2), "write_s": round(wrote, 3),
                "threads": host_threads(), "bit_identical_to_values": same,
                "note": "mmap + threads, Clinger's fast path, strtod otherwise (fscanf's values); "
                        "the reference's fscanf reads the same file token by token"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def exact_kernel_name(eng) -> str:
    """The exact kernel shard 0 runs: over its column-panel copy, or the row-major dispatch."""
    from matvec_mpi_multiplier_amd._lib import lib

    sh = eng.shard(0)
    P = eng.exact_panel_width(0)
    if P:
        v = lib.mvg_gemv_exact_panel_auto_variant(sh.n_rows, sh.n_cols)
        return f"{lib.mvg_gemv_exact_panel_variant_name(v).decode()} (column panels, P = {P})"
    name = lib.mvg_gemv_exact_variant_name(lib.mvg_gemv_exact_auto_variant(sh.n_cols, sh.n_rows, sh.n_cols)).decode()
    dev = int(os.environ.get("LOCAL_RANK", "0")) if os.environ.get("MVG_SAME_DEVICE") != "1" else 0
    if lib.mvg_gemv_exact_even_refused(dev) == 1:  # the runtime turned down the evenly placed form here
        name += " (evenly placed form refused by the runtime: one-wave forms)"
    return name


# BASELINE.json configs[2..4], each at its own fixed size (strong scaling over N); the GPU
# counts BASELINE.json quotes each one at ("across 1/2/4/8", "2x4 GPU grid", "at 8 GPUs")
BASELINE_CONFIGS = [
    ("config 3", "colwise", 65536, 65536),
    ("config 4", "blockwise", 131072, 131072),
    ("config 5", "rowwise", 4194304, 512),
]
DEFINED_AT = {3: (1, 2, 4, 8), 4: (8,), 5: (8,)}


def config_order(spec: str, n: int) -> list[int]:
    """The configs the section runs, in order. An explicit list ("3,4,5") is kept as given;
    "auto" puts the configs BASELINE.json defines at this N first, highest number first (at
    N = 8: 5, 4, 3 — config 5 is the one defined only at 8 GPUs), then the others by per-GPU
    bytes, smallest first (N = 1: 3, 5, 4)."""
    if spec.strip() != "auto":
        return [int(k) for k in spec.split(",") if k.strip()]
    by_num = {int(c[0].split()[-1]): c for c in BASELINE_CONFIGS}
    defined = sorted((k for k in by_num if n in DEFINED_AT[k]), reverse=True)
    rest = sorted((k for k in by_num if k not in defined), key=lambda k: by_num[k][2] * by_num[k][3])
    return defined + rest


def config_passes(args, n, rank, budget, report, run_device, run_e2e, run_cpu, headline_e2e=None,
                  headline_bytes=0):
    """BASELINE configs 3-5 in three passes, so that no end-to-end loop can cost a config its
    device-resident number (round 5: the /dev/shm setup of configs 3 and 4 at N = 8 left no
    budget for config 5):
      1. every config's device-resident tree and exact steps, in config_order (run_device(k) ->
         (entry, y): the entry goes into the line at once, y stays here for the later passes);
      2. the end-to-end loops, smallest A first: the headline's (headline_e2e(), into the line's
         `end_to_end`) and each config's in --config-e2e that has a device-resident y
         (run_e2e(k, y) -> its `end_to_end`);
      3. at N = 1, each config's CPU baseline (run_cpu(k, y) -> its `cpu_baseline`).
    The passes' order and every skip are the same on every rank (run_* decide collectively).
    Returns {k: entry}."""
    by_num = {int(c[0].split()[-1]): c for c in BASELINE_CONFIGS}
    entries, ys = {}, {}
    for k in config_order(args.configs, n) if not args.no_configs else []:
        entry, y = run_device(k)
        entries[k] = entry
        if isinstance(entry, dict) and "value" in entry:
            ys[k] = y
        if rank == 0:
            report.append("configs", entry)
    e2e_set = {int(k) for k in args.config_e2e.split(",") if k.strip()}
    jobs = []  # (bytes of A, order, what)
    if headline_e2e is not None:
        jobs.append((headline_bytes, 0, None))
    for k in ys:
        name, alg, R, C = by_num[k]
        if k in e2e_set:
            jobs.append((8 * R * C, k, k))
        with report.lock:
            entries[k]["end_to_end"] = ({"pending": "the end-to-end pass, after every config's device-resident steps"}
                                        if k in e2e_set else "not requested (--config-e2e)")
    if not args.no_e2e and args.e2e_iters > 0:
        for _, _, k in sorted(jobs, key=lambda j: (j[0], j[1])):
            if k is None:
                got = headline_e2e()
                if rank == 0:
                    report["end_to_end"] = got
                continue
            got = run_e2e(k, ys[k])
            with report.lock:
                entries[k]["end_to_end"] = got
    if n == 1 and rank == 0 and not args.no_cpu_baseline and not args.no_config_cpu_baseline:
        for k in ys:
            got = run_cpu(k, ys[k])
            with report.lock:
                entries[k]["cpu_baseline"] = got
    return entries


def config_device(args, mm, comm, n, rank, local, distributed, barrier, budget, guarded, k):
    """Pass 1 for config k on the N GPUs: its shard must fit in free HBM on every rank (decided
    collectively, like the budget) and its estimate in the budget; then one_config. Returns
    (entry, y on rank 0 or None)."""
    import torch
    import torch.distributed as dist

    name, alg, R, C = {int(c[0].split()[-1]): c for c in BASELINE_CONFIGS}[k]
    try:
        sh = mm.plan_shard(alg, R, C, n, rank)
    except mm.IndivisibleError as exc:  # the same on every rank: no collective is entered
        return {"config": name, "alg": alg, "R": R, "C": C, "skipped": f"does not split over {n} GPUs: {exc}"}, None
    part = R if alg == "colwise" else sh.y_len
    need = 8 * (sh.n_rows * sh.n_cols + sh.n_cols + (9 + n) * part + R) + (1 << 30)  # + exact-mode gather buffer
    free = torch.cuda.mem_get_info(local)[0]
    ok = torch.tensor([1.0 if free >= need else 0.0], dtype=torch.float64, device=f"cuda:{local}")
    if distributed:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if float(ok[0]) < 1.0:
        return {"config": name, "alg": alg, "R": R, "C": C, "skipped": f"needs {need >> 30} GiB of HBM per GPU"}, None
    per = 8 * (sh.n_rows * sh.n_cols + sh.n_cols + part)
    got = budget.run(name, est_config(per, args.config_steps), guarded, one_config, args, mm, comm, n, rank,
                     local, distributed, barrier, name, alg, R, C)
    if isinstance(got, tuple):
        return got
    return {"config": name, "alg": alg, "R": R, "C": C, **(got if isinstance(got, dict) else {})}, None


def config_e2e(args, mm, comm, n, rank, local, distributed, barrier, budget, guarded, k, y):
    """Pass 2 for config k: north_star's end-to-end time — the root's host A distributed over
    every GPU's link, multiplied, y on the root (the reference's timing semantics) — on a fresh
    engine, wherever host memory (and /dev/shm at N > 1) holds A, measured now; y must equal
    the device-resident y of pass 1 bit for bit (same values, same kernels)."""
    name, alg, R, C = {int(c[0].split()[-1]): c for c in BASELINE_CONFIGS}[k]
    total = sum(8 * (s.n_rows * s.n_cols + s.n_cols + (R if alg == "colwise" else s.y_len))
                for s in (mm.plan_shard(alg, R, C, n, r) for r in range(n)))
    fit, mem = e2e_memory_fit(R, C, distributed, local, cap=int(args.host_mem_cap_gib * 2 ** 30))
    if not fit:
        return {"skipped": "memory", **mem}

    def run():
        e = mm.Multiplier(alg, R, C, comm)
        try:
            return end_to_end(args, e, mm, R, C, rank, distributed, barrier, y, total, local, budget)
        finally:
            e.destroy()

    got = budget.run(f"{name} end_to_end", est_e2e(total, n, args.e2e_iters, distributed), guarded, run)
    if isinstance(got, dict):
        got.setdefault("host_memory", {}).update(mem)
    return got


def config_cpu(args, budget, guarded, k, y):
    """Pass 3 for config k (rank 0, N = 1): the reference on a leading-row slice at the host's
    core count, and the -O2 port on the whole config where host memory allows (config 4: its
    leading rows), each checked against the device-resident y."""
    name, alg, R, C = {int(c[0].split()[-1]): c for c in BASELINE_CONFIGS}[k]
    ref_rows = min(R, max(128, int(args.config_ref_bytes // (8 * C))))
    return budget.run(
        f"{name} cpu_baseline",
        est_cpu_baseline(args, R, C, ref_rows=ref_rows, sweep=False, port_bytes=args.config_cpu_sample_bytes,
                         cpu_seconds=args.config_cpu_seconds, placements=1),
        guarded, cpu_baseline, args, alg, R, C, y, None, ref_rows, args.config_cpu_sample_bytes,
        args.config_cpu_seconds, ("spread",), (), None, collective=False)


def one_config(args, mm, comm, n, rank, local, distributed, barrier, name, alg, R, C):
    """One BASELINE config's device-resident steps on the N GPUs (pass 1 of config_passes):
    tree-mode steps, then the bit-exact steps; on rank 0 its y against the reference's own rows.
    Returns (entry, y)."""
    import torch
    import torch.distributed as dist

    sh = mm.plan_shard(alg, R, C, n, rank)
    part = R if alg == "colwise" else sh.y_len

    def timed(e, steps):
        e.kernel_timing(args.event_every)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            e.multiply()
        e.sync()
        barrier()
        el = time.perf_counter() - t0
        kt = e.kernel_ms()
        e.kernel_timing(0)
        by_rank[0] = per_rank(kt.avg_ms, distributed, local)
        t = torch.tensor([el, kt.avg_ms], dtype=torch.float64, device=f"cuda:{local}")
        if distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0]), float(t[1])

    by_rank = [None]
    total = sum(8 * (s.n_rows * s.n_cols + s.n_cols + (R if alg == "colwise" else s.y_len))
                for s in (mm.plan_shard(alg, R, C, n, r) for r in range(n)))
    per = 8 * (sh.n_rows * sh.n_cols + sh.n_cols + part)
    exact = None
    e = mm.Multiplier(alg, R, C, comm)
    try:
        e.fill_synth()
        vram_wait = wait_vram_cleared(local)  # the previous config's engine was just freed
        warm(e, 3, distributed, local)
        el, kms = timed(e, args.config_steps)
        tree_by_rank = by_rank[0]
        y = e.collect()
        yx = None
        if rank == 0:
            expect(np.all(np.isfinite(y)) and y.min() >= 0.0 and y.max() <= C * 0.9999 ** 2, f"{name}: y out of range")
        if not args.no_exact:
            # the same config in bit-exact mode: exact kernels + the exact exchange (gather of
            # every partial to rank 0, the reference's combine order there)
            e.set_exact(True)
            warm(e, 2, distributed, local)
            xsteps = max(5, args.config_steps // 2)
            xel, xkms = timed(e, xsteps)
            yx = e.collect()
            xkernel = exact_kernel_name(e)
            e.set_exact(False)
            exact = {"value": round(total * xsteps / xel / 1e9, 1), "ms_per_step": round(xel / xsteps * 1e3, 4),
                     "gflops": round(2 * R * C * xsteps / xel / 1e9, 1),
                     "steps": xsteps, "kernel": xkernel, "kernel_ms": round(xkms, 5),
                     "kernel_ms_by_rank": by_rank[0], "pmc": pmc_summary(sh.n_rows, sh.n_cols, xkernel),
                     "kernel_frac": round(per / (xkms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if xkms > 0 else None}
            if rank == 0:
                rel = float(np.max(np.abs(yx - y) / np.abs(y)))
                expect(rel <= 1e-12, f"{name}: exact y differs from the tree-summed y by {rel}")
                exact["max_rel_vs_tree"] = rel
    finally:
        e.destroy()
    gr, gcols = mm.get_2_most_closest_multipliers(n)
    entry = {
        "config": name, "alg": alg, "R": R, "C": C, "shard": [sh.n_rows, sh.n_cols],
        "grid": [gr, gcols] if alg == "blockwise" else None,
        "value": round(total * args.config_steps / el / 1e9, 1), "unit": "GB/s",
        "ms_per_step": round(el / args.config_steps * 1e3, 4), "steps": args.config_steps,
        "gflops": round(2 * R * C * args.config_steps / el / 1e9, 1),
        "kernel": kernel_name(sh), "kernel_ms": round(kms, 5), "kernel_ms_by_rank": tree_by_rank,
        "kernel_frac": round(per / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if kms > 0 else None,
        "pmc": pmc_summary(sh.n_rows, sh.n_cols, kernel_name(sh)),
        "exact": exact,
        "vram_wait": vram_wait,
    }
    if rank == 0:
        entry["reference_rows"] = reference_rows_check(name, alg, R, C, n, y, yx)
    return entry, (y if rank == 0 else None)


def host_mem_free() -> int:
    """Host bytes this process may still take: MemAvailable, capped by its cgroup's memory.max
    less memory.current when a limit is set (the GPU pool's per-command cap)."""
    free = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                free = int(line.split()[1]) * 1024
    except OSError:
        pass
    try:
        lim = open("/sys/fs/cgroup/memory.max").read().strip()
        if lim != "max":
            cap = int(lim) - int(open("/sys/fs/cgroup/memory.current").read().strip())
            free = cap if free is None else min(free, cap)
    except (OSError, ValueError):
        pass
    return max(0, free or 0)


def process_rss() -> int:
    try:
        for line in open("/proc/self/status"):
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def e2e_memory_fit(R, C, distributed, local, margin=8 << 30, cap=None):
    """Whether the end-to-end loop's host copy of A (R x C fp64; in /dev/shm at N > 1, a
    process's own memory at N = 1) fits with `margin` and 5 % to spare, on every rank (MIN):
    within the host memory measured now and, with `cap`, within cap less this process's RSS."""
    import torch
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd.hostshare import shm_free_bytes

    need = 8 * R * C
    free = host_mem_free()
    if cap is not None:
        free = min(free, max(0, cap - process_rss()))
    shm = shm_free_bytes() if distributed else None
    ok = free >= need * 1.05 + margin and (shm is None or shm >= need + (1 << 30))
    if distributed:
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = float(t[0]) >= 1.0
    return ok, {"need_bytes": need, "host_free_bytes": free, "shm_free_bytes": shm}


SLICES = os.path.join(REPO, "tests", "golden", "config_slices.npz")


def reference_rows_check(name, alg, R, C, n, y, yx):
    """The config's y on the rows the real reference computed at the same (R, C, P = n)
    (tests/golden/config_slices.npz: oracle/_ref under mpiexec -n P on four bands of the config's
    rows, which is the reference's y for those rows of the full problem). Tree form: <= 1e-12
    (asserted); exact form: bit-identical except the block split over more than two grid columns,
    whose reference sum follows message arrival order."""
    key_cfg = "cfg" + name.split()[-1]
    if not os.path.exists(SLICES):
        return None
    with np.load(SLICES) as z:
        key = f"{key_cfg}/{alg}/P{n}"
        if key not in z.files and alg == "rowwise" and f"{key_cfg}/{alg}/P1" in z.files:
            key = f"{key_cfg}/{alg}/P1"  # a row's sum does not depend on P (matr_utils.c:86-96)
        if key not in z.files:
            return {"P": n, "checked": False, "why": f"no reference slice for P = {n}"}
        rows, want = z[f"{key_cfg}/rows"], z[key]
    rel = float(np.max(np.abs(y[rows] - want) / np.abs(want)))
    expect(rel <= 1e-12, f"{name}: y differs from the reference's own y on its rows by {rel}")
    out = {"P": n, "rows": int(len(rows)), "max_rel": rel,
           "source": "tests/golden/config_slices.npz: oracle/_ref, mpiexec -n P, on 4 bands of the config's rows"
                     + ("" if key.endswith(f"/P{n}") else f" (reference run at {key.split('/')[-1]}: row sums do not depend on P)")}
    if yx is not None:
        grid_cols = mm_grid_cols(n) if alg == "blockwise" else 1
        out["exact_bit_identical"] = bool(np.array_equal(yx[rows], want))
        out["exact_max_rel"] = float(np.max(np.abs(yx[rows] - want) / np.abs(want)))
        if grid_cols > 2:
            out["exact_note"] = "grid of > 2 columns: the reference adds in message-arrival order"
    return out


def mm_grid_cols(n):
    from matvec_mpi_multiplier_amd import multiplier as mm

    return mm.get_2_most_closest_multipliers(n)[1]


def parse_rccl_log(lines):
    """RCCL's NCCL_DEBUG=INFO lines -> {"links": {"a->b": [transport, ...]}, "nranks": [...],
    "samples": [...]}: the transport of every connection it set up ("Channel 00/0 : 0[0] -> 1[1]
    via P2P/IPC", "... [send] via NET/Socket/0") and the size of every communicator it reports
    initialised ("... nranks 8 ... Init COMPLETE")."""
    import re

    pat = re.compile(r"(\d+)\[\w+\] -> (\d+)\[\w+\](?: \[(?:send|receive)\])? via (\S+)")
    links, nranks, samples = {}, [], []
    for line in lines:
        m = pat.search(line)
        if m:
            links.setdefault(f"{m.group(1)}->{m.group(2)}", set()).add(m.group(3))
            if len(samples) < 2:
                samples.append(line.strip()[-160:])
        m = re.search(r"nranks (\d+)", line)
        if m and "Init COMPLETE" in line:
            nranks.append(int(m.group(1)))
    return {"links": {k: sorted(v) for k, v in links.items()}, "nranks": nranks, "samples": samples}


def rccl_warnings(lines):
    """The WARN / ERROR lines of an RCCL log ("host:pid:tid [dev] NCCL WARN ...")."""
    return [ln.rstrip() for ln in lines if " NCCL WARN " in ln or " NCCL ERROR " in ln]


def per_rank(ms, distributed, local):
    """Every rank's mean GEMV time (ms), in rank order (None at N = 1): the max over ranks is the
    step's kernel time, the spread shows whether one GPU lags the others."""
    if not distributed:
        return None
    import torch
    import torch.distributed as dist

    t = torch.tensor([ms], dtype=torch.float64, device=f"cuda:{local}")
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [round(float(v[0]), 5) for v in out]


def rccl_report(path, distributed, rank):
    """What RCCL reported about its communicators, all ranks gathered on rank 0: the transport of
    every connection it set up ("a->b": P2P/IPC, P2P/direct pointer, SHM, NET/...), counted per
    transport, and the communicator sizes (nranks) it initialised. Parsed from the NCCL_DEBUG=INFO
    file each rank wrote (its WARN / ERROR lines go on to stderr); {"logged": false, ...} when the
    caller set NCCL_DEBUG_FILE (RCCL then logs where the caller asked, untouched)."""
    import torch.distributed as dist

    mine = {"links": {}, "nranks": [], "samples": []}
    if path and os.path.exists(path):
        with open(path, errors="replace") as f:
            lines = f.readlines()
        mine = parse_rccl_log(lines)
        for line in rccl_warnings(lines):  # what a caller's NCCL_DEBUG=WARN would have shown
            log(line)
        try:
            os.remove(path)
        except OSError:
            pass
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, mine)
    if rank != 0:
        return None
    if path is None:
        return {"logged": False, "why": "NCCL_DEBUG_FILE set by the caller"}
    links, counts, sizes, samples = {}, {}, set(), []
    for r in allr:
        sizes.update(r["nranks"])
        samples += r["samples"][: max(0, 4 - len(samples))]
        for k, v in r["links"].items():
            links.setdefault(k, set()).update(v)
    for v in links.values():
        for t in v:
            counts[t] = counts.get(t, 0) + 1
    return {"logged": True, "comm_sizes": sorted(sizes), "transport_counts": counts,
            "links": {k: sorted(v) for k, v in sorted(links.items())}, "log_samples": samples}


def end_to_end(args, eng, mm, R, C, rank, distributed, barrier, y_ref, total_bytes, local, budget=None):
    """The reference's timing semantics on the GPU path: A and x preloaded in the root's host
    memory; each iteration distributes them, multiplies, and ends when the root holds y (max over
    ranks). Two distributions:
      shared    : the root's A lives in host shared memory every rank maps; each GPU pulls its own
                  shard over its own PCIe link, all at once (MPICH's shared-memory scatter analog;
                  N = 1: one process, plain pinned memory).
      root_send : only the root touches A; it stages each peer's shard through its GPU and
                  ncclSends it over xGMI (the reference's sequential root sends). N > 1 only.
    With a `budget`, an iteration after the first runs only if 1.5x the slowest one so far still
    fits (all-reduced), and root_send only if (N - 1)x the shared form's iteration does — the
    root pushes N - 1 shards through its one link — so a slow transport (the same-device
    rehearsal's sockets) costs at most one iteration beyond the budget; `iters` says how many ran."""
    import torch
    import torch.distributed as dist

    from matvec_mpi_multiplier_amd._lib import lib as _l

    def timed(fn):
        times = []
        for it in range(args.e2e_iters):
            if it > 0 and budget is not None and not budget.fits(1.5 * max(times)):
                break
            barrier()
            ts = time.perf_counter()
            y = fn()
            barrier()
            tt = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=f"cuda:{local}")
            if distributed:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            times.append(float(tt[0]))
        if rank == 0:
            expect(np.array_equal(y, y_ref), "end-to-end y differs from the device-resident y")
        out_t = {"mean_s": float(np.mean(times)), "iters": len(times),
                 "GBps": total_bytes / float(np.mean(times)) / 1e9,
                 "gflops": 2 * R * C / float(np.mean(times)) / 1e9}
        if len(times) < args.e2e_iters:
            out_t["stopped"] = "budget"
        return out_t

    out = {"semantics": "reference: root holds A, x in host memory; distribute + multiply + y on root"}
    from matvec_mpi_multiplier_amd.hostshare import SharedHostMatrix, shm_free_bytes

    from matvec_mpi_multiplier_amd.hostshare import fill_threads

    shared = None
    setup = {}  # this rank's host-matrix setup: fill (first touch) and page-locking, timed apart
    t_fill = time.perf_counter()
    if not distributed:
        A = mm.synth_host(R, C, 42)
        setup.update(rows=R, threads=host_threads(), fill_s=round(time.perf_counter() - t_fill, 3))
    else:
        local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", str(n_ranks(distributed))))
        shared = SharedHostMatrix.create(R, C, 42, f"bench_{os.environ.get('MASTER_PORT', '0')}",
                                         device=f"cuda:{local}", threads=fill_threads(local_ranks))
        A = shared.array if shared is not None else None
        if shared is not None:
            setup.update(shared.timing)
        if shared is None:
            out["shared"] = f"skipped: /dev/shm has {shm_free_bytes() >> 30} GiB free, needs {(R * C * 8) >> 30} GiB"
    x = mm.synth_host(1, C, 4242)[0]
    have_shared = A is not None
    if distributed and not have_shared and rank == 0:
        A = mm.synth_host(R, C, 42)  # root-only copy for the root_send distribution
    # page-lock what this rank's GPU reads: all of A on the root (it also stages every peer's shard
    # for root_send) and at N = 1; a peer's own rows otherwise (its row block's lines; the column
    # split's strip spans every row)
    reg = None
    if A is not None:
        sh = eng.shard(0)
        if distributed and rank != 0 and eng.name != "colwise":
            reg = host_rows_region(A, sh.row_off, sh.row_off + sh.n_rows)
        else:
            reg = (A.ctypes.data, A.nbytes)
        t_pin = time.perf_counter()
        if _l.mvg_host_register(*reg) != 0:
            reg = None
        setup.update(pin_bytes=reg[1] if reg else 0, pin_s=round(time.perf_counter() - t_pin, 3))
    pinned = reg is not None
    out["host_memory"] = host_setup_record(setup, distributed, C)
    if have_shared:
        out["shared"] = timed(lambda: (eng.distribute_shared(A, x), eng.multiply(), eng.collect())[2])
        out["shared"]["distribution"] = ("per-GPU H2D from " + ("shared " if distributed else "")
                                         + ("pinned" if pinned else "pageable") + " host memory")
    if distributed:
        per = out["shared"]["mean_s"] if isinstance(out.get("shared"), dict) else 8 * R * C / 20e9
        need = 1.5 * max(1, n_ranks(distributed) - 1) * per
        if budget is not None and not budget.fits(need):
            out["root_send"] = budget.marker(need)
        else:
            out["root_send"] = timed(lambda: (eng.distribute(A if rank == 0 else None, x), eng.multiply(),
                                              eng.collect())[2])
            out["root_send"]["distribution"] = "root H2D staging + ncclSend over xGMI"
    if pinned:
        _l.mvg_host_unregister(reg[0])
    if shared is not None:
        eng._keep = None
        del A
        shared.close()
    # the bound of this path is the GPU's host link, not HBM: report it as a roofline of its own
    # (per-GPU rate of the slowest rank against the link's spec and a plain pinned H2D copy)
    link = pcie_roofline(local)
    if link is not None:
        best = min((v["mean_s"] for v in (out.get("shared"), out.get("root_send")) if isinstance(v, dict) and "mean_s" in v),
                   default=None)
        if best is not None:
            per_gpu = total_bytes / n_ranks(distributed) / best / 1e9
            link["achieved"] = round(per_gpu, 2)
            link["frac"] = round(per_gpu / link["peak"], 4) if link.get("peak") else None
            link["frac_of_copy"] = round(per_gpu / link["h2d_copy_GBps"], 4)
        out["roofline"] = link
    return out


def host_setup_record(mine, distributed, C):
    """Every rank's host-matrix setup (rows filled, fill threads, fill and page-lock seconds),
    gathered to rank 0, with the aggregate rates: the fill's bytes over the slowest rank's fill,
    the page-locked bytes over the slowest rank's hipHostRegister."""
    allr = [mine]
    if distributed:
        import torch.distributed as dist

        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, mine)
    rec = {"by_rank": allr}
    rows = sum(r.get("rows", 0) for r in allr if r)
    fill = max((r.get("fill_s", 0.0) for r in allr if r), default=0.0)
    pin = max((r.get("pin_s", 0.0) for r in allr if r), default=0.0)
    pinned = sum(r.get("pin_bytes", 0) for r in allr if r)
    return {**rec, "fill_s": fill, "pin_s": pin, "pin_bytes": pinned,
            "rows": rows, "fill_GBps": round(8 * rows * C / fill / 1e9, 2) if fill > 0 else None,
            "pin_GBps": round(pinned / pin / 1e9, 2) if pin > 0 else None}


def host_rows_region(A, r0, r1, page=4096):
    """(address, bytes) of rows [r0, r1) of the row-major host matrix A, widened to whole pages
    within A's buffer (page-locking works on pages)."""
    row = A.shape[1] * A.itemsize
    base, end = A.ctypes.data, A.ctypes.data + A.nbytes
    lo = max(base, (base + r0 * row) // page * page)
    hi = min(end, -(-(base + r1 * row) // page) * page)
    return lo, max(0, hi - lo)


def n_ranks(distributed):
    import torch.distributed as dist

    return dist.get_world_size() if distributed else 1


def pcie_roofline(local):
    """The host link of GPU `local`: its PCIe generation and width from sysfs (peak = the
    per-direction payload rate after 128b/130b line coding) and the rate of a plain 1 GiB
    page-locked host -> device copy on it (HIP events), the practical ceiling of distribution."""
    import torch

    out = {"bound": "pcie", "unit": "GB/s"}
    try:
        p = torch.cuda.get_device_properties(local)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        base = f"/sys/bus/pci/devices/{bdf}"
        speed = open(f"{base}/current_link_speed").read().strip()  # e.g. "32.0 GT/s PCIe"
        width = int(open(f"{base}/current_link_width").read().strip())
        gts = float(speed.split()[0])
        out.update({"link": f"{speed} x{width}", "pci": bdf,
                    "peak": round(gts * width * (128 / 130) / 8, 2) if gts >= 8 else None})
    except Exception as exc:  # sysfs layout differs: keep the measured ceiling only
        out.update({"link": f"unknown ({type(exc).__name__})", "peak": None})
    try:
        n = 1 << 27  # 1 GiB of fp64
        h = torch.empty(n, dtype=torch.float64, pin_memory=True)
        h.fill_(1.0)
        d = torch.empty(n, dtype=torch.float64, device=f"cuda:{local}")
        s = torch.cuda.Stream(device=f"cuda:{local}")
        best = None
        with torch.cuda.stream(s):
            for _ in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                d.copy_(h, non_blocking=True)
                e1.record(s)
                e1.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
        out["h2d_copy_GBps"] = round(8 * n / (best * 1e-3) / 1e9, 2)
        del h, d
    except Exception as exc:
        log(f"pcie_roofline: copy probe failed: {exc}")
        return None
    return out


def cpu_baseline(args, alg, R, C, y_gpu, y_exact=None, ref_rows=None, sample_bytes=None, cpu_seconds=None,
                 placements=("spread", "compact"), sweep_ps=(), big_rows=None):
    """The reference's CPU path timed on this host. Preferred: the real reference (oracle/_ref,
    built from its own sources, run with MPICH's mpiexec on P = the port's thread count) on the
    leading rows of the same matrix, kind "reference"; its 100-iteration loop is fixed in its
    source. Always also: the oracle port (below), reported under "port" (or as the baseline
    itself, kind "port", when the reference cannot run here).

    Two samples. The small one (`ref_rows` rows) picks the placement (the port's spread CPUs or
    consecutive cores: the reference is communication-bound, its root scatters A through MPI
    shared memory every iteration) and carries the rank sweep `sweep_ps` (`sweep`: time, GB/s,
    speed-up and efficiency as its README defines them, S = T1 / TP and E = S / P,
    README.md:47-50). With `big_rows`, the reference then runs on a sample at least twice the
    last-level cache of the CPUs it uses (`host_cache`, from sysfs) at P and at P = 1 on the
    winning placement, and that beyond-cache run is the baseline's `value`; the small sample's
    figures stay under `small_sample`."""
    ref_rows = args.ref_rows if ref_rows is None else ref_rows
    port = cpu_port_baseline(args, alg, R, C, y_gpu, y_exact, sample_bytes, cpu_seconds)
    if args.no_ref_baseline:
        return port
    from oracle import cpuset, ref_runner

    P = port["cores"]
    cpus = port["placement"]["cpus"]
    rows = splittable_rows(alg, min(R, ref_rows), P)
    if not ref_runner.available(alg) or not _splits(alg, rows, C, P):
        port["reference"] = "not run: oracle/_ref or mpiexec absent, or the sample does not split"
        return port
    runs = []
    sets = {"spread": cpus, "compact": None}
    for label in placements:
        cset = sets[label] if sets[label] is not None else cpuset.pick_compact(P, gpu_numa_node())
        try:
            runs.append((label, cset, ref_runner.run(alg, rows, C, P, timeout=args.ref_timeout, cpus=cset, track=CHILDREN,
                                                     rows=np.arange(rows))))
        except Exception as exc:  # the baseline must never sink the bench
            port.setdefault("reference_errors", []).append(f"{label}: {str(exc)[:200]}")
    if not runs:
        port["reference"] = "not run: " + "; ".join(port.get("reference_errors", []))
        return port
    label, cpus, r = min(runs, key=lambda t: t[2]["seconds"])
    by_placement = {lab: round(8 * (rows * C + C + rows) / rr["seconds"] / 1e9, 3) for lab, _, rr in runs}
    rel = float(np.max(np.abs(y_gpu[:rows] - r["y"]) / np.abs(r["y"])))
    expect(rel <= 1e-12, f"GPU y differs from the reference's own y: {rel}")
    nbytes = 8 * (rows * C + C + rows)
    sweep = ref_sweep(args, alg, rows, C, P, r["seconds"], label, sweep_ps, nbytes) if sweep_ps else None
    cache = host_cache(cpus)

    def sample_text(nrows, rr, relv):
        return (f"leading {nrows} of {R} rows ({nrows}x{C}, {8 * nrows * C / 2 ** 20:.0f} MiB) {alg}: the "
                f"reference's own executable (oracle/_ref, MPICH mpiexec -n {P}, gcc -O0 as its test.sh) on its "
                f"text inputs, its 100-iteration loop (distribution from the root + sequential sums + "
                f"collection); run {rr['wall_s']:.1f} s incl. text loading; GPU y matches its y to {relv:.1e}")

    small = {"value": round(nbytes / r["seconds"] / 1e9, 3), "ms_per_step": round(r["seconds"] * 1e3, 3),
             "rows": rows, "bytes": nbytes, "sample": sample_text(rows, r, rel)}
    out = {"value": small["value"], "unit": "GB/s", "cores": P, "kind": "reference", "sweep": sweep,
           "ms_per_step": small["ms_per_step"], "iters": 100, "sample": small["sample"],
           "host_cpu": host_cpu(), "host_cache": cache,
           "placement": {**cpuset.describe(cpus), "kind": label, "GBps_by_placement": by_placement},
           "port": {k: port[k] for k in ("value", "ms_per_step", "cores", "sample")},
           "exact_vs_port": port.get("exact_vs_port"),
           **({"exact_vs_reference": bool(np.array_equal(y_exact[:rows], r["y"]))}
              if y_exact is not None and alg == "rowwise" else {})}
    l3 = (cache or {}).get("l3_bytes")
    l3s = (cache or {}).get("l3_bytes_system")
    # the sample against the L3 of the CPUs the ranks run on, and against the host's whole L3
    out["sample_over_l3"] = round(nbytes / l3, 2) if l3 else None
    out["sample_over_l3_system"] = round(nbytes / l3s, 2) if l3s else None
    if big_rows:
        brows = splittable_rows(alg, min(R, big_rows), P)
        if brows <= rows:
            out["big_sample"] = f"not run: {brows} rows is not beyond the small sample"
        else:
            bbytes = 8 * (brows * C + C + brows)
            try:
                rb = ref_runner.run(alg, brows, C, P, timeout=args.ref_timeout, cpus=cpus, rows=np.arange(brows),
                                    track=CHILDREN)
                relb = float(np.max(np.abs(y_gpu[:brows] - rb["y"]) / np.abs(rb["y"])))
                expect(relb <= 1e-12, f"GPU y differs from the reference's own y (beyond-cache sample): {relb}")
                pts = [{"P": P, "s_per_iter": round(rb["seconds"], 6), "GBps": round(bbytes / rb["seconds"] / 1e9, 3)}]
                if P > 1 and 1 in sweep_ps:
                    try:
                        r1 = ref_runner.run(alg, brows, C, 1, timeout=args.ref_timeout, track=CHILDREN,
                                            cpus=cpuset.pick(1, gpu_numa_node()), rows=np.arange(brows))
                        pts.insert(0, {"P": 1, "s_per_iter": round(r1["seconds"], 6),
                                       "GBps": round(bbytes / r1["seconds"] / 1e9, 3)})
                    except Exception as exc:  # a sweep point must never sink the bench
                        out["big_sample_errors"] = [f"P=1: {str(exc)[:160]}"]
                t1 = pts[0]["s_per_iter"] if pts[0]["P"] == 1 else None
                for pt in pts:
                    pt["speedup"] = round(t1 / pt["s_per_iter"], 3) if t1 else None
                    pt["efficiency"] = round(t1 / pt["s_per_iter"] / pt["P"], 3) if t1 else None
                out.update(value=round(bbytes / rb["seconds"] / 1e9, 3), ms_per_step=round(rb["seconds"] * 1e3, 3),
                           sample=sample_text(brows, rb, relb), sample_over_l3=round(bbytes / l3, 2) if l3 else None,
                           sample_over_l3_system=round(bbytes / l3s, 2) if l3s else None,
                           sweep_beyond_cache={"points": pts, "semantics": "the same executable on the beyond-cache "
                                               "sample; S = T1/TP, E = S/P (README.md:47-50)"},
                           small_sample=small)
                if y_exact is not None and alg == "rowwise":
                    out["exact_vs_reference"] = bool(np.array_equal(y_exact[:brows], rb["y"]))
            except Exception as exc:  # the small sample's figures stand
                out["big_sample"] = f"failed: {str(exc)[:300]}"
    return out


def splittable_rows(alg, rows, P):
    """`rows` rounded down to what the algorithm splits over P ranks (a multiple of the ranks
    over rows: P for the row split, the grid's rows for the block split)."""
    if alg in ("rowwise", "blockwise"):
        from oracle import oracle

        gr = P if alg == "rowwise" else oracle.grid_shape(P)[0]
        rows = max(gr, rows - rows % gr)
    return rows


def big_sample_rows(args, alg, R, C, factor=2.0, min_bytes=1 << 30):
    """Rows of the beyond-cache CPU sample: at least `factor` x the host's last-level cache
    (all of it, every instance: the reference's ranks may run anywhere in the quota) and at least
    1 GiB of A, at most the whole matrix."""
    cache = host_cache(None) or {}
    need = max(min_bytes, factor * (cache.get("l3_bytes_system") or 0))
    return int(min(R, -(-int(need) // (8 * C))))


def host_cache(cpus=None):
    """The last-level (L3) cache from sysfs for the CPUs `cpus` (default: every CPU of the host):
    size of one instance, the distinct instances those CPUs use, and their total (`l3_bytes`);
    `l3_bytes_system`: all instances on the host. None when sysfs has no L3."""
    base = "/sys/devices/system/cpu"

    def size_bytes(txt):
        txt = txt.strip()
        mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(txt[-1:], 1)
        return int(txt.rstrip("KMG")) * mult

    try:
        inst = {}
        for path in glob.glob(f"{base}/cpu[0-9]*/cache/index*/level"):
            if open(path).read().strip() != "3":
                continue
            d = os.path.dirname(path)
            cpu = int(d.split("/cpu")[-1].split("/")[0])
            shared = open(f"{d}/shared_cpu_list").read().strip()
            inst.setdefault(shared, [size_bytes(open(f"{d}/size").read()), set()])[1].add(cpu)
        if not inst:
            return None
        used = [v for v in inst.values() if cpus is None or v[1] & set(cpus)]
        return {"l3_instance_bytes": max(v[0] for v in inst.values()), "l3_instances": len(used),
                "l3_bytes": sum(v[0] for v in used), "l3_bytes_system": sum(v[0] for v in inst.values()),
                "source": f"{base}/cpu*/cache/index*/ (level 3)"}
    except (OSError, ValueError):
        return None


def ref_sweep(args, alg, rows, C, P, seconds_at_P, label_at_P, ps, nbytes):
    """The real reference on the same leading-rows sample at each rank count in `ps` (and at P,
    already run): mpiexec -n p, confined to p CPUs of the GPU's NUMA node first (oracle/cpuset),
    its own 100-iteration loop. The reference's scaling sweep is `mpiexec -n $np` over np in
    {1, 2, 6, 12, 24} (test.sh:5-11); speed-up S = T1 / TP, efficiency E = S / P
    (README.md:47-50). Rank counts that do not split the sample are skipped."""
    from oracle import cpuset, ref_runner

    times, where, errors = {P: seconds_at_P}, {P: label_at_P}, []
    for p in sorted(set(ps)):
        if p == P or p > P or p < 1 or not _splits(alg, rows, C, p):
            continue
        try:
            rr = ref_runner.run(alg, rows, C, p, timeout=args.ref_timeout, cpus=cpuset.pick(p, gpu_numa_node()), track=CHILDREN,
                                rows=np.arange(rows))
            times[p], where[p] = rr["seconds"], "spread"
        except Exception as exc:  # a sweep point must never sink the bench
            errors.append(f"P={p}: {str(exc)[:160]}")
    t1 = times.get(1)
    pts = [{"P": p, "s_per_iter": round(t, 6), "GBps": round(nbytes / t / 1e9, 3),
            "speedup": round(t1 / t, 3) if t1 else None, "efficiency": round(t1 / t / p, 3) if t1 else None,
            "placement": where[p]} for p, t in sorted(times.items())]
    return {"points": pts, "errors": errors or None,
            "semantics": "the reference's own executable on the sample above, mpiexec -n P; S = T1/TP, E = S/P "
                         "(README.md:47-50)"}


def cpu_port_baseline(args, alg, R, C, y_gpu, y_exact=None, sample_bytes=None, cpu_seconds=None):
    """The oracle restatement of the reference's CPU path (P threads as MPI ranks, distribution
    from the root's A included, mean of per-iteration max) on this host, on the full workload
    or, above `sample_bytes`, on its leading rows (same values, same algorithm)."""
    from matvec_mpi_multiplier_amd import multiplier as mm
    from oracle import oracle

    sample_bytes = args.cpu_sample_bytes if sample_bytes is None else sample_bytes
    cpu_seconds = args.cpu_seconds if cpu_seconds is None else cpu_seconds
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    rows = R
    if R * C * 8 > sample_bytes:
        rows = max(1, int(sample_bytes // (C * 8)))
    # keep the sample splittable the way the algorithm splits it over `threads` ranks: sampled
    # rows are rounded down to a multiple of the ranks over rows; the column split (fixed C)
    # lowers the rank count instead
    if rows < R and alg in ("rowwise", "blockwise"):
        gr = oracle.grid_shape(threads)[0] if alg == "blockwise" else threads
        rows = max(gr, rows - rows % gr)
    while threads > 1 and not _splits(alg, rows, C, threads):
        threads -= 1
    # the inputs (not the timed path): the library's threaded generator of the same values
    A = mm.synth_host(rows, C, 42)
    x = oracle.synth(1, C, 4242)[0]
    # `cores` is enforced, not assumed: the port's threads (and the reference's ranks after it)
    # run confined to exactly `threads` CPUs, those of the GPU's NUMA node first
    from oracle import cpuset

    cpus = cpuset.pick(threads, gpu_numa_node())
    threads = len(cpus)
    with cpuset.confined(cpus):
        t1, y_cpu = oracle.time_multiply(alg, A, x, threads, 1)
        iters = max(2, min(200, int(cpu_seconds / max(t1, 1e-6))))
        t, y_cpu = oracle.time_multiply(alg, A, x, threads, iters)
    del A
    rel = float(np.max(np.abs(y_gpu[:rows] - y_cpu) / np.abs(y_cpu)))
    expect(rel <= 1e-12, f"GPU y differs from the reference restatement: {rel}")
    exact_same = None
    if y_exact is not None and alg == "rowwise":
        # row sums do not depend on the rank count, so the port's P-rank y is the reference's y
        # for the GPU's single shard too; the exact mode must reproduce it bit for bit (the
        # column and block splits' combine orders depend on P, and the GPU runs P = N here)
        exact_same = bool(np.array_equal(y_exact[:rows], y_cpu))
        expect(exact_same, "exact-mode y differs from the reference restatement")
    nbytes = 8 * (rows * C + C + rows)
    what = "full workload" if rows == R else f"sample: leading {rows} of {R} rows"
    return {"exact_vs_port": exact_same, "value": round(nbytes / t / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "ms_per_step": round(t * 1e3, 3), "iters": iters,
            "sample": f"{what} ({rows}x{C}) {alg}, {threads} threads as ranks, {iters} iterations "
                      f"(reference timing semantics: distribution from the root's A + sequential sums + "
                      f"collection, max over ranks; gcc -O2); GPU y matches to {rel:.1e}",
            "host_cpu": host_cpu(), "placement": {"cpus": cpus, "record": cpuset.describe(cpus)}}


def gpu_numa_node():
    from matvec_mpi_multiplier_amd._lib import lib
    import ctypes

    node = ctypes.c_int(-1)
    try:
        dev = int(os.environ.get("LOCAL_RANK", "0"))
        if lib.mvg_device_numa_node(dev, ctypes.byref(node)) == 0 and node.value >= 0:
            return node.value
    except Exception:  # placement is best effort; the CPU count is enforced either way
        pass
    return None


def _splits(alg, R, C, p):
    if alg == "rowwise":
        return R % p == 0
    if alg == "colwise":
        return C % p == 0
    from oracle import oracle

    gr, gc = oracle.grid_shape(p)
    return C % gc == 0 and R >= gr


def kernel_name(sh) -> str:
    from matvec_mpi_multiplier_amd._lib import lib

    return lib.mvg_gemv_variant_name(lib.mvg_gemv_auto_variant(sh.n_cols, sh.n_rows, sh.n_cols)).decode()


def host_cpu():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
