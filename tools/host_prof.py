#!/usr/bin/env python3
"""The host side of one main-line search on a machine without a GPU: libtsg's host code built
over tests/sanitize/host_stub.cpp (`make -C tests/sanitize prof`), whose stand-in device returns
about as many matches as the bench's config-2 query finds (one entry in TSG_STUB_ONE_IN) with no
device time (TSG_STUB_SLEEP_US=0). What is left per search_raw step is what the host adds around
the device: tsg_search's planning, the coalescer, the result assembly, ctypes.

    make -C tests/sanitize prof && python3 tools/host_prof.py [--steps 3000] [--blocks 10]
"""
import argparse
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "build", "san", "prof", "lib", "libtsg.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--blocks", type=int, default=10)
    ap.add_argument("--entries", type=int, default=1_000_000)
    ap.add_argument("--one-in", type=int, default=19500)  # ~513 matches over 10 M entries
    ap.add_argument("--workdir", default="/tmp/tsg_host_prof")
    a = ap.parse_args()
    if os.environ.get("TSG_LIB_PATH") != LIB:  # (the library is chosen at import: a child with the env)
        env = dict(os.environ, TSG_LIB_PATH=LIB, TSG_STUB_DEVICES="1", TSG_STUB_SLEEP_US="0", TSG_STUB_CACHE="1",
                   TSG_STUB_ONE_IN=str(a.one_in))
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))
    sys.path.insert(0, ROOT)
    import tempo_amd as T
    sys.path.insert(0, ROOT)
    import bench
    os.makedirs(a.workdir, exist_ok=True)
    paths = bench.gen_blocks(a.workdir, 0, a.blocks, a.entries, 8)
    eng = T.Engine()
    blocks = tuple(eng.open_block(p) for p in paths)
    pipe = T.Pipeline(T.SearchRequest(**bench.QUERY))
    n, _ = eng.search_raw(blocks, pipe, metrics=False)
    for _ in range(200):
        eng.search_raw(blocks, pipe, metrics=False)
    ts = []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        eng.search_raw(blocks, pipe, metrics=False)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print("matches %d  step us: p10 %.2f p50 %.2f p90 %.2f mean %.2f" % (
        n, ts[len(ts) // 10] * 1e6, ts[len(ts) // 2] * 1e6, ts[len(ts) * 9 // 10] * 1e6, sum(ts) / len(ts) * 1e6))
    for b in blocks:
        b.close()


if __name__ == "__main__":
    main()
