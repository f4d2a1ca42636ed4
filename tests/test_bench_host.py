"""Host-side helpers of bench.py (no GPU): CPU placement picks whole cores."""
import os

import bench


def _core(c):
    try:
        return open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
    except OSError:
        return str(c)


def test_idlest_picks_distinct_cores():
    cpus = sorted(os.sched_getaffinity(0))
    k = min(4, len(cpus))
    got = bench.idlest(cpus, k, window=0.05)
    assert len(got) == k and len(set(got)) == k and set(got) <= set(cpus)
    ncores = len({_core(c) for c in cpus})
    if ncores >= k:  # one CPU per core whenever there are enough cores
        assert len({_core(c) for c in got}) == k


def test_idlest_fills_when_cores_are_few():
    cpus = sorted(os.sched_getaffinity(0))[:2]
    got = bench.idlest(cpus, 2, window=0.01)
    assert sorted(got) == sorted(cpus)
