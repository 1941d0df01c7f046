"""CPU placement of the CPU baselines (oracle/cpuset.py): spread over physical cores and L3
domains, confinement restores the affinity."""
import os

from oracle import cpuset


def test_spread_round_robins_l3_domains_and_defers_smt_siblings(monkeypatch):
    # 2 CCDs x 2 cores x 2 threads: cpu c on core c % 4, CCD (c % 4) // 2; siblings c and c + 4
    def key(c, what):
        if what.startswith("topology"):
            return f"core{c % 4}"
        return f"l3-{(c % 4) // 2}"

    monkeypatch.setattr(cpuset, "_cpu_key", key)
    order = cpuset._spread(list(range(8)))
    assert order[:4] == [0, 2, 1, 3]          # one per physical core, CCDs alternating
    assert sorted(order[4:]) == [4, 5, 6, 7]  # SMT siblings last
    assert sorted(order) == list(range(8))


def test_pick_and_confined_restore_affinity():
    before = os.sched_getaffinity(0)
    cpus = cpuset.pick(2)
    assert 1 <= len(cpus) <= 2 and set(cpus) <= before
    with cpuset.confined(cpus):
        assert os.sched_getaffinity(0) == set(cpus)
    assert os.sched_getaffinity(0) == before
    d = cpuset.describe(cpus)
    assert d["cpus_allowed"] == len(before) and "cgroup_quota" in d
