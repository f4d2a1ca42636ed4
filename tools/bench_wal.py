#!/usr/bin/env python3
"""WAL search blocks (StreamingSearchBlock): replay + search
throughput of one synthetic search WAL file on the GPU, the oracle's replay + search
of the same file on the host beside it, and a parity check of the two.

Prints one JSON line (not the bench.py headline): entries/s of a resident-block
search (the replay is timed separately, as the reference replays once at startup).
"""
import argparse
import json
import os
import random
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gen(path, n, seed, dup_frac):
    import tempo_amd as T
    rng = random.Random(seed)
    t0 = 1_700_000_000 * 10**9
    ents = []
    for i in range(n):
        tid = rng.getrandbits(128).to_bytes(16, "big")
        start = t0 + rng.randrange(3600 * 10**9)
        e = {"id": tid, "start": start, "end": start + int(rng.lognormvariate(17.7, 1.5)),
             "tags": {"service.name": "svc-%02d" % rng.randrange(40), "http.method": rng.choice(["get", "post", "put"]),
                      "status.code": str(rng.choice([0, 1, 1, 1, 2])), "http.url": "/api/v1/users/%d" % rng.randrange(500),
                      "root.service.name": "svc-%02d" % rng.randrange(40), "root.name": "op-%d" % rng.randrange(30)}}
        ents.append(e)
        if rng.random() < dup_frac:  # the same trace appended again (a later batch of spans)
            ents.append({"id": tid, "start": start + 1000, "end": e["end"] + 10**6,
                         "tags": {"db.statement": "select * from t%d" % rng.randrange(50)}})
    rng.shuffle(ents)
    T.write_wal_search(path, ents, T.ENC_SNAPPY)
    return len(ents)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, default=200_000)
    ap.add_argument("--dup", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    import tempo_amd as T
    from oracle import oracle as O

    d = tempfile.mkdtemp(prefix="tsg_wal_", dir="/tmp")
    try:
        path = os.path.join(d, T.wal_filename(T.ENC_SNAPPY))
        t = time.time()
        pages = gen(path, args.entries, 7, args.dup)
        gen_s = time.time() - t
        eng = T.Engine(devices=[0])
        t = time.perf_counter()
        blk = eng.open_wal_block(path)
        replay_s = time.perf_counter() - t
        info = blk.info()
        q = dict(tags={"service.name": "svc-07", "http.method": "get"}, min_duration_ms=10, max_duration_ms=1000)
        pipe = T.Pipeline(T.SearchRequest(**q))
        got, met = eng.search([blk], pipe)
        for _ in range(5):
            eng.search_raw([blk], pipe)
        t = time.perf_counter()
        for _ in range(args.steps):
            eng.search_raw([blk], pipe)
        step_s = (time.perf_counter() - t) / args.steps
        ob = O.Block(path, wal=True)
        t = time.perf_counter()
        exp, omet, st = O.search([ob], tags=q["tags"], min_ms=10, max_ms=1000)
        cpu_s = time.perf_counter() - t
        parity = st == 0 and [(m.entry_idx, m.trace_id) for m in got] == [(m["entry_idx"], m["id"]) for m in exp] \
            and met.inspected_traces == omet["traces_inspected"] and met.inspected_bytes == omet["bytes_inspected"]
        print(json.dumps({
            "metric": "WAL search entries/s (StreamingSearchBlock, resident)", "value": info["entries"] / step_s,
            "unit": "entries/s", "entries": info["entries"], "wal_pages": pages, "matches": len(got),
            "step_us": step_s * 1e6, "replay_s": replay_s, "gen_s": gen_s,
            "cpu_baseline": {"value": info["entries"] / cpu_s, "unit": "entries/s", "cores": 1, "kind": "port",
                             "sample": "oracle replay + dedupe/combine + StreamingSearchBlock.Search of the same file, "
                                       "one thread (the reference replays once; this includes it)"},
            "parity": parity}), flush=True)
        blk.close()
        eng.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
