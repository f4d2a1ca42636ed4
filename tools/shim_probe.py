#!/usr/bin/env python3
"""The bench's shim leg alone (config-2 set, 10 C threads x 1 block per query), one limit per
process, so TSG_PROF's per-phase percentiles (printed at exit) belong to that limit only."""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--limit", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--workdir", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import tempo_amd as T
    wd = a.workdir or tempfile.mkdtemp(prefix="shimprobe_", dir="/tmp")
    paths = bench.gen_blocks(wd, 0, 10, a.entries, 10)
    eng = T.Engine(devices=[0])
    base = bench.parallel(eng.open_block, paths)
    sets = [base] + [[b.clone(eng) for b in base] for _ in range(3)]
    q = bench.QUERY
    pipe = T.Pipeline(T.SearchRequest(tags=q["tags"], min_duration_ms=q["min_duration_ms"],
                                      max_duration_ms=q["max_duration_ms"], start=q["start"], end=q["end"]))
    node = eng.numa_node(0)
    cpus = bench.node_cpus(node) & os.sched_getaffinity(0) if node >= 0 else set()
    if len(cpus) > 12:
        os.sched_setaffinity(0, set(bench.idlest(sorted(cpus), 12)))
    eng.shim_pattern(sets, pipe, 16, limit=a.limit)
    t0 = time.time()
    ns, nm = eng.shim_pattern(sets, pipe, a.rounds, limit=a.limit)
    slow = [(i, x / 1e3) for i, x in enumerate(ns) if x > 1e6]
    print({"limit": a.limit, "query_us": bench.pct([x / 1e3 for x in ns]), "records": sorted(set(nm)),
           "slow_rounds": slow[:20], "wall_s": time.time() - t0}, flush=True)
    for s in sets:
        for b in s:
            b.close()
    eng.close()


if __name__ == "__main__":
    main()
