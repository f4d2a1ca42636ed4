#!/usr/bin/env python3
"""One rank of the limit-over-ranks check on the GPU (tests/test_gpu_limit_ranks.py starts
`--nproc-per-node N` of these under torch.distributed.run). Every rank opens its range of
the blocks on the device and runs tempo_amd.shard.distributed_search_limit over a gloo group
with Engine.search_wire / Engine.cancel; rank 0 also runs ONE tsg_search(limit=L) over all
blocks and writes whether the two agree record for record and in the metrics, and the
records and metrics themselves (the test checks them against the oracle's consumer)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", nargs="+", required=True)
    ap.add_argument("--limit", type=int, required=True)
    ap.add_argument("--tags", default="{}")
    ap.add_argument("--min-ms", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch.distributed as dist
    dist.init_process_group("gloo")
    import tempo_amd as T
    from tempo_amd import shard
    rank, world = dist.get_rank(), dist.get_world_size()
    eng = T.Engine(devices=[0])
    try:
        pipe = T.Pipeline(T.SearchRequest(tags=json.loads(a.tags), min_duration_ms=a.min_ms))
        mine = [eng.open_block(a.blocks[i]) for i in shard.shard_range(len(a.blocks), world, rank)]
        res = shard.distributed_search_limit(
            lambda seen, qid: eng.search_wire(mine, pipe, limit=a.limit, query_id=qid, seen=seen),
            eng.cancel, a.limit, query_id=7000 + rank)
        if rank == 0:
            allb = [eng.open_block(p) for p in a.blocks]
            one = shard.from_wire(eng.search_wire(allb, pipe, limit=a.limit))
            # records compared field by field with names resolved (the name tables are laid out per rank)
            recs = lambda r: [(bytes(x["trace_id"]), int(x["start_ns"]), int(x["duration_ms"]),  # noqa: E731
                               r.name(x["root_service"]), r.name(x["root_name"])) for x in r.recs]
            met = lambda r: (r.metrics.inspected_traces, r.metrics.inspected_bytes,  # noqa: E731
                             r.metrics.inspected_blocks, r.metrics.skipped_blocks)
            ok = recs(res) == recs(one) and met(res) == met(one)
            # the records themselves (the test compares them with the oracle's consumer)
            out = [[r[0].hex(), r[1], r[2], r[3].decode("utf-8", "replace") if isinstance(r[3], bytes) else r[3],
                    r[4].decode("utf-8", "replace") if isinstance(r[4], bytes) else r[4]] for r in recs(res)]
            with open(a.out, "w") as f:
                json.dump({"ok": bool(ok), "n": len(res), "n_one": len(one), "metrics": met(res),
                           "metrics_one": met(one), "records": out}, f)
            for b in allb:
                b.close()
        for b in mine:
            b.close()
    finally:
        eng.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
