#!/usr/bin/env python3
"""Kernel time of the search launch for query shapes around config 2 (diagnostics).

Generates (or reuses --workdir) the config-2 block set, then for each query shape
prints the average HIP-event kernel time and the algorithmic bytes. With
TSG_STAMPS=1 libtsg also prints per-phase workgroup timestamps per search.
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

T0 = 1_700_000_000
SHAPES = {
    "cfg2": dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"},
                 min_duration_ms=10, max_duration_ms=1000, start=T0 + 900, end=T0 + 2700),
    "dur_range": dict(min_duration_ms=10, max_duration_ms=1000, start=T0 + 900, end=T0 + 2700),
    "range": dict(start=T0 + 900, end=T0 + 2700),
    "tags3": dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"}),
    "tag1": dict(tags={"service.name": "svc-07"}),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10)
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    import bench
    import tempo_amd as T
    work = tempfile.mkdtemp(prefix="tsg_probe_", dir="/tmp")
    paths = bench.gen_blocks(work, 0, args.blocks, args.entries, 16)
    eng = T.Engine(devices=[0])
    blocks = [eng.open_block(p) for p in paths]
    for name in args.shapes.split(","):
        q = SHAPES[name]
        pipe = T.Pipeline(T.SearchRequest(**q))
        for _ in range(3):
            eng.search_raw(blocks, pipe, flags=T.SEARCH_TIME_SCAN)
        ns = []
        for _ in range(args.reps):
            n, met = eng.search_raw(blocks, pipe, flags=T.SEARCH_TIME_SCAN)
            ns.append(met.scan_kernel_ns)
        avg = sum(ns) / len(ns)
        print(json.dumps({"shape": name, "matches": n, "kernel_us": avg / 1e3, "min_us": min(ns) / 1e3,
                          "scan_bytes": met.scan_bytes, "gbps": met.scan_bytes / avg}), flush=True)
    for b in blocks:
        b.close()
    eng.close()


if __name__ == "__main__":
    main()
