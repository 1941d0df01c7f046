"""The reference's CPU path on this host at several rank counts (P = 1/2/4/8 and the
host's core share), beside the oracle's threaded port — TEST/BENCH INFRASTRUCTURE.

    python tools/cpu_ref_sweep.py [--rows 1024] [--cols 16384] [--procs 1,2,4,8,16]

Runs oracle/_ref (the reference built from its own sources, MPICH mpiexec) on the leading
`rows` rows of config 2's matrix (same synthetic values, the reference's "%.4f" text), its fixed
100-iteration loop, and the port (oracle/cpu_ref.c, P threads as ranks) on the same sample.
Prints one JSON line per (alg, P) with the per-iteration time and the GB/s of A, plus a header
line describing the host (lscpu model, cores visible to this process).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cpuset, oracle, ref_runner  # noqa: E402


def host():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"host_cpu": model, "cpus_visible": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_quota": cpuset.cgroup_cpu_quota(),
            "binding": "each (alg, P) run confined to P CPUs (sched_setaffinity on mpiexec, inherited by "
                       "its ranks; the port's P threads likewise); 'cpuset' per line"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--cols", type=int, default=16384)
    ap.add_argument("--procs", default="1,2,4,8,16")
    ap.add_argument("--algs", default="rowwise,colwise,blockwise")
    args = ap.parse_args()
    print(json.dumps(host()), flush=True)
    R, C = args.rows, args.cols
    A = oracle.synth_block(0, R, 0, C, C, 42)
    x = oracle.synth(1, C, 4242)[0]
    nbytes = 8 * R * C
    for alg in args.algs.split(","):
        for P in (int(p) for p in args.procs.split(",")):
            cpus = cpuset.pick(P)
            line = {"alg": alg, "R": R, "C": C, "P": P, "cpuset": cpuset.describe(cpus)["cpuset"]}
            try:
                r = ref_runner.run(alg, R, C, P, timeout=900, cpus=cpus)
                line.update(ref_ms=round(r["seconds"] * 1e3, 3), ref_GBps=round(nbytes / r["seconds"] / 1e9, 3),
                            ref_wall_s=round(r["wall_s"], 1))
                y_ref = r["y"]
            except Exception as exc:  # an indivisible P or a missing launcher: say so, go on
                line["ref_error"] = str(exc)[:200]
                y_ref = None
            try:
                with cpuset.confined(cpus):
                    t, y = oracle.time_multiply(alg, A, x, P, 20)
                line.update(port_ms=round(t * 1e3, 3), port_GBps=round(nbytes / t / 1e9, 3))
                if y_ref is not None:
                    line["port_vs_ref_max_rel"] = float(abs(y - y_ref).max() / abs(y_ref).max())
            except ValueError as exc:  # P does not split this sample for this algorithm
                line["port_error"] = str(exc)
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
