"""Where the N > 1 end-to-end setup's time goes: the host matrix's first-touch fill and its
page-locking (hipHostRegister), timed apart, per process, for P processes that each own R/P rows
(the bench's ranks), in private anonymous memory or in one /dev/shm segment (hostshare.py), with
T fill threads per process. One JSON line per (mode, P, T). Development probe (MI355X box).

    python tools/probes/host_setup_probe.py [GiB] [modes] [P list] [T list]
    e.g. python tools/probes/host_setup_probe.py 32 anon,shm,shm_falloc 1,4 16,4

Modes: anon (each process its own numpy rows), shm (one segment, first touch by the fill),
shm_falloc (each process posix_fallocate's its own byte range of the segment first, so the
pages exist before the fill writes them), shm_populate (madvise(MADV_POPULATE_WRITE) on its
range first), shm_pinfirst (hipHostRegister on its untouched range first — the kernel allocates
the pages while pinning — then the fill writes pinned pages), shm_perrank (each process its own
segment for its rows: an MPI-3 shared window's per-rank segments; one tmpfs file per process).
T = 0: the 16-CPU quota split over the P processes.
"""
import json
import os
import sys
import time
from multiprocessing import get_context

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
C = 16384


def worker(args):
    mode, name, R, P, p, T, q = args
    os.environ["MVG_THREADS"] = str(T or max(1, 16 // P))
    os.environ["MVG_NO_TORCH"] = "1"
    sys.path.insert(0, REPO)
    import mmap

    import numpy as np

    from matvec_mpi_multiplier_amd._lib import check, lib

    r0, r1 = R * p // P, R * (p + 1) // P
    out = {"p": p, "rows": r1 - r0}
    t = time.perf_counter()
    if mode == "anon":
        A = np.empty((r1 - r0, C))
        base, nb, keep = A.ctypes.data, A.nbytes, A
    elif mode == "shm_perrank":
        size = (r1 - r0) * C * 8
        fd = os.open(f"/dev/shm/{name}_{p}", os.O_CREAT | os.O_RDWR, 0o600)
        os.ftruncate(fd, size)
        m = mmap.mmap(fd, size)
        os.close(fd)
        os.unlink(f"/dev/shm/{name}_{p}")  # the mapping keeps it until the process ends
        A = np.ndarray((r1 - r0, C), buffer=m)
        base, nb, keep = A.ctypes.data, A.nbytes, (m, A)
    else:
        fd = os.open(f"/dev/shm/{name}", os.O_RDWR)
        size = R * C * 8
        if mode == "shm_falloc":
            os.posix_fallocate(fd, r0 * C * 8, (r1 - r0) * C * 8)
        m = mmap.mmap(fd, size)
        os.close(fd)
        A = np.ndarray((R, C), buffer=m)[r0:r1]
        base, nb, keep = A.ctypes.data, A.nbytes, (m, A)
        if mode == "shm_populate":
            m.madvise(23, r0 * C * 8, (r1 - r0) * C * 8)  # MADV_POPULATE_WRITE
    pin_first = mode == "shm_pinfirst"
    if pin_first:
        rc = lib.mvg_host_register(base, nb)
        out["pin_rc"] = rc
    out["alloc_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    check(lib.mvg_synth_fill_host(base, C, r1 - r0, C, r0, 0, C, 42), "fill")
    out["fill_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    if not pin_first:
        rc = lib.mvg_host_register(base, nb)
        out["pin_rc"] = rc
    out["pin_s"] = round(time.perf_counter() - t, 3)
    if rc == 0:
        t = time.perf_counter()
        lib.mvg_host_unregister(base)
        out["unpin_s"] = round(time.perf_counter() - t, 3)
    del A, keep
    q.put(out)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 32
    modes = (sys.argv[2] if len(sys.argv) > 2 else "anon,shm,shm_falloc").split(",")
    Ps = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,4").split(",")]
    Ts = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "16,4").split(",")]
    R = int(gib * 2 ** 30 / (8 * C))
    ctx = get_context("spawn")
    info = {}
    for path in ("/sys/kernel/mm/transparent_hugepage/shmem_enabled", "/sys/kernel/mm/transparent_hugepage/enabled",
                 "/proc/sys/vm/nr_hugepages", "/sys/fs/cgroup/cpu.max"):
        try:
            info[path] = open(path).read().strip()
        except OSError as exc:
            info[path] = f"unreadable: {exc}"
    info["cpus_affinity"] = len(os.sched_getaffinity(0))
    print(json.dumps({"host": info}), flush=True)
    for mode in modes:
        for P in Ps:
            for T in Ts:
                name = f"mvg_probe_{os.getpid()}"
                if mode not in ("anon", "shm_perrank"):
                    fd = os.open(f"/dev/shm/{name}", os.O_CREAT | os.O_RDWR, 0o600)
                    os.ftruncate(fd, R * C * 8)
                    os.close(fd)
                q = ctx.Queue()
                t = time.perf_counter()
                procs = [ctx.Process(target=worker, args=((mode, name, R, P, p, T, q),)) for p in range(P)]
                for pr in procs:
                    pr.start()
                res = [q.get(timeout=600) for _ in procs]
                for pr in procs:
                    pr.join()
                wall = time.perf_counter() - t
                if mode not in ("anon", "shm_perrank"):
                    os.unlink(f"/dev/shm/{name}")
                nb = R * C * 8
                fill = max(r["fill_s"] + r["alloc_s"] for r in res)
                pin = max(r["pin_s"] for r in res)
                total = max(r["fill_s"] + r["alloc_s"] + r["pin_s"] for r in res)
                rate = (lambda s: round(nb / s / 1e9, 2) if s > 0 else None)  # noqa: E731
                print(json.dumps({"mode": mode, "P": P, "T": T, "GiB": gib, "wall_s": round(wall, 2),
                                  "fill_GBps": rate(fill), "pin_GBps": rate(pin), "setup_GBps": rate(total),
                                  "per_process": sorted(res, key=lambda r: r["p"])}), flush=True)


if __name__ == "__main__":
    main()
