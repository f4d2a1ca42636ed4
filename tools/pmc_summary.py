#!/usr/bin/env python3
"""Per-launch HBM-side traffic of the search kernels from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are kilobytes at the L2's memory side (Infinity Cache
hits included). On gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads (MI355X_MICROARCH.md, HBM section), so reads are doubled.
Usage: pmc_summary.py <FETCH_SIZE run dir> <WRITE_SIZE run dir> [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", help="merge into this JSON file (profiles/pmc_traffic.json) under --workload")
    ap.add_argument("--workload", default="blocks=10,entries=1000000")
    ap.add_argument("--source", default="", help="where the passes came from (recorded next to the numbers)")
    ap.add_argument("--match", default="search,prep,dict", help="kernel name substrings to report (comma list)")
    args = ap.parse_args()
    fetch = per_kernel(args.fetch_dir, "FETCH_SIZE")
    write = per_kernel(args.write_dir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not any(m in k for m in args.match.split(",")):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        # skip the first (full-result) search of the bench; average the rest
        f2, w2 = (f[1:] or f), (w[1:] or w)
        rd = 2 * 1024 * sum(f2) / len(f2) if f2 else None
        wr = 1024 * sum(w2) / len(w2) if w2 else None
        out[k] = {"launches": len(f), "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "traffic_bytes_per_launch": (rd or 0) + (wr or 0)}
    print(json.dumps(out, indent=1))
    if args.out:
        try:
            with open(args.out) as f:
                merged = json.load(f)
        except (OSError, ValueError):
            merged = {}
        for k in out:
            out[k]["source"] = args.source
        w = merged.setdefault(args.workload, {})
        w.update(out)  # (other kernels measured on this workload keep their entries)
        w["_source"] = args.source
        with open(args.out, "w") as f:
            json.dump(merged, f, indent=1)


if __name__ == "__main__":
    main()
