"""CPU placement for the CPU baselines — TEST/BENCH INFRASTRUCTURE ONLY.

The CPU baseline reports `cores`; this module makes that number a fact rather than a thread
count: the reference's MPI ranks (oracle/ref_runner.py) and the port's threads (oracle/oracle.py)
run with their affinity confined to exactly that many CPUs, and the record carries the CPU list
and the job's cgroup CPU quota (how many CPUs' worth of time the scheduler grants, whatever
os.cpu_count() says on a shared host).
"""
from __future__ import annotations

import contextlib
import os


def cgroup_cpu_quota() -> dict:
    """{"cpus": quota / period or None (unlimited), "source": file} from cgroup v2 cpu.max or
    v1 cpu.cfs_quota_us / cpu.cfs_period_us; {"cpus": None, "source": None} if neither reads."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return {"cpus": None if q == "max" else round(int(q) / int(p), 2), "source": "/sys/fs/cgroup/cpu.max",
                "raw": f"{q} {p}"}
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return {"cpus": None if q < 0 else round(q / p, 2), "source": "/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
                "raw": f"{q} {p}"}
    except (OSError, ValueError):
        return {"cpus": None, "source": None}


def _node_cpus(node: int) -> set[int]:
    out: set[int] = set()
    try:
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    except (OSError, ValueError):
        pass
    return out


def _cpu_key(c: int, what: str) -> str:
    try:
        return open(f"/sys/devices/system/cpu/cpu{c}/{what}").read().strip()
    except OSError:
        return str(c)


def _spread(cpus: list[int]) -> list[int]:
    """Order `cpus` so that the first k of them sit on k different physical cores spread
    round-robin over the L3 domains (CCDs): a memory-bound CPU baseline on n CPUs then gets the
    bandwidth of as many CCDs as it can reach, not of the one or two that n consecutive CPU
    numbers share. SMT siblings come after every physical core."""
    seen_core: set[str] = set()
    primary, siblings = [], []
    for c in cpus:
        core = _cpu_key(c, "topology/thread_siblings_list")
        (siblings if core in seen_core else primary).append(c)
        seen_core.add(core)
    domains: dict[str, list[int]] = {}
    for c in primary:
        domains.setdefault(_cpu_key(c, "cache/index3/shared_cpu_list"), []).append(c)
    rr, lists = [], list(domains.values())
    for i in range(max((len(v) for v in lists), default=0)):
        rr.extend(v[i] for v in lists if i < len(v))
    return rr + siblings


def pick(n: int, numa_node: int | None = None) -> list[int]:
    """n CPUs from this process's affinity set: those of `numa_node` first (the GPU's node, so
    the baseline and the GPU share a socket), then the rest; within each group one CPU per
    physical core, spread over the L3 domains (`_spread`). Fewer if fewer exist."""
    allowed = sorted(os.sched_getaffinity(0))
    node = _node_cpus(numa_node) if numa_node is not None else set()
    first = [c for c in allowed if c in node]
    rest = [c for c in allowed if c not in node]
    return (_spread(first) + _spread(rest))[:max(1, n)]


def pick_compact(n: int, numa_node: int | None = None) -> list[int]:
    """n CPUs on consecutive physical cores (SMT siblings last), those of `numa_node` first: the
    placement that suits a communication-bound run (MPI ranks exchanging through shared memory
    stay on few L3 domains), where `pick` suits a bandwidth-bound one."""
    allowed = sorted(os.sched_getaffinity(0))
    node = _node_cpus(numa_node) if numa_node is not None else set()

    def primary_first(cpus):
        seen, first, later = set(), [], []
        for c in cpus:
            core = _cpu_key(c, "topology/thread_siblings_list")
            (later if core in seen else first).append(c)
            seen.add(core)
        return first + later

    first = primary_first([c for c in allowed if c in node])
    return (first + primary_first([c for c in allowed if c not in node]))[:max(1, n)]


@contextlib.contextmanager
def confined(cpus: list[int]):
    """Confine this process (and the threads it starts meanwhile) to `cpus`; restore after."""
    before = os.sched_getaffinity(0)
    os.sched_setaffinity(0, cpus)
    try:
        yield
    finally:
        os.sched_setaffinity(0, before)


def describe(cpus: list[int]) -> dict:
    return {"cpuset": _ranges(cpus), "cpus_allowed": len(os.sched_getaffinity(0)),
            "os_cpu_count": os.cpu_count(), "cgroup_quota": cgroup_cpu_quota()}


def _ranges(cpus: list[int]) -> str:
    cpus = sorted(cpus)
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)
