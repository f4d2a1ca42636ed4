#!/usr/bin/env python3
"""Per-launch HBM-side traffic of the search kernels from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are kilobytes at the L2's memory side (Infinity Cache
hits included). On gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads (MI355X_MICROARCH.md, HBM section), so reads are doubled.
Usage: pmc_summary.py <FETCH_SIZE run dir> <WRITE_SIZE run dir>
"""
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
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if "search" not in k and "prep" not in k:
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


if __name__ == "__main__":
    main()
