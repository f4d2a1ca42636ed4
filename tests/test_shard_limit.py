"""Limit queries over ranks (tempo_amd.shard.distributed_search_limit), on the CPU (gloo).

SURVEY.md §8(e): with limit L each rank searches its block range with its own early exit;
the ranks' distinct IDs are consumed in rank order on rank 0, the rank where the consumer
reaches L searches again with the IDs before it (tsg_search_opts.seen_ids), ranks after it
are cancelled. The merged result must be exactly what ONE sequential consumer over all
blocks in order returns (instance_search.go:45-60): the same records in the same order and
the same metrics (blocks / traces / bytes inspected up to where it stops).

Without a GPU the rank's search is the oracle (test-side stand-in for Engine.search_wire:
orc_search_seeded is the same consumer started with the IDs taken before); what is under
test is the protocol in tempo_amd.shard. tests/test_gpu_limit_ranks.py runs it on the GPU.
"""
import os
import random
import socket
import tempfile
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
import tempo_amd as T
from tempo_amd import shard
from helpers import random_entries, write_block

QUERY = dict(tags={"k1": "v1"}, min_ms=5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make_blocks(tmpdir, nblocks=6, n=300, dense=()):
    rng = random.Random(17)
    paths = []
    for b in range(nblocks):
        ents = random_entries(rng, n)
        if b % 2:  # ids repeated across blocks: a duplicate counts once toward L
            ents[:30] = [dict(e) for e in random_entries(random.Random(99), 30)]
            ents.sort(key=lambda e: e["id"])
        if b not in dense:  # sparse blocks: few k1=v1 matches
            for e in ents[20:]:
                e["tags"].pop("k1", None)
        paths.append(write_block(tmpdir, f"b{b}", ents))
    return paths


def oracle_wire(blocks, limit, seen):
    got, met, st = O.search(blocks, limit=limit, seen=seen, **QUERY)
    assert st == 0
    traces = [T.TraceSearchMetadata(trace_id=m["id"], trace_id_len=m["id_len"],
                                    root_service_name=m["root_service"].decode(),
                                    root_trace_name=m["root_name"].decode(), start_time_unix_nano=m["start_ns"],
                                    duration_ms=m["duration_ms"]) for m in got]
    sm = T.SearchMetrics(met["traces_inspected"], met["bytes_inspected"], met["blocks_inspected"],
                         met["blocks_skipped"], block_status=met["block_status"], block_errors=[None] * len(blocks))
    return shard.to_wire(shard.response_from_traces(traces, sm))


def key(resp):
    r = resp.recs
    return ([(bytes(r["trace_id"][i]), int(r["start_ns"][i]), int(r["duration_ms"][i]), resp.name(r["root_service"][i]),
              resp.name(r["root_name"][i])) for i in range(len(r))],
            (resp.metrics.inspected_traces, resp.metrics.inspected_bytes, resp.metrics.inspected_blocks,
             resp.metrics.skipped_blocks))


def _worker(rank, world, port, paths, limit, slow_rank, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = [O.Block(paths[i]) for i in shard.shard_range(len(paths), world, rank)]
        state = {"cancelled": False, "searches": 0}

        def search(seen, qid):
            state["searches"] += 1
            if rank == slow_rank and seen is None:  # a slow rank: the drop must cancel it
                for _ in range(400):
                    if state["cancelled"]:
                        raise T.TsgError(T.TSG_E_CANCELLED, "search cancelled (tsg_cancel)")
                    time.sleep(0.01)
            return oracle_wire(mine, limit, seen)

        def cancel(qid):
            state["cancelled"] = True

        res = shard.distributed_search_limit(search, cancel, limit, query_id=1000 + rank)
        with open(os.path.join(outdir, f"state{rank}.txt"), "w") as f:
            f.write("%d %d" % (state["cancelled"], state["searches"]))
        if rank == 0:
            np.save(os.path.join(outdir, "wire.npy"), shard.to_wire(res))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


def run(paths, world, limit, slow_rank=-1):
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, _free_port(), paths, limit, slow_rank, td), nprocs=world, join=True)
        res = shard.from_wire(np.load(os.path.join(td, "wire.npy")))
        states = [tuple(int(x) for x in open(os.path.join(td, f"state{r}.txt")).read().split()) for r in range(world)]
        return res, states


def expected(paths, limit):
    return shard.from_wire(oracle_wire([O.Block(p) for p in paths], limit, None))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("limit", [0, 5, 40, 10_000])
def test_limit_over_ranks_equals_one_consumer(tmp_path, world, limit):
    """Sparse blocks: the stop lands in rank 0, in a later rank, or nowhere (every match).
    limit 0 is "every match" (as in tsg_search): no rank is a stop point."""
    paths = _make_blocks(str(tmp_path))
    got, _ = run(paths, world, limit)
    exp = expected(paths, limit)
    assert key(got) == key(exp) and len(got) > 0


def test_stop_in_rank0_cancels_a_slow_rank(tmp_path):
    """Dense first blocks: rank 0 alone reaches L; a rank still searching is told to drop and
    cancels (tsg_cancel), and the result is still the single consumer's."""
    paths = _make_blocks(str(tmp_path), dense=(0, 1))
    got, states = run(paths, 3, 20, slow_rank=2)
    assert key(got) == key(expected(paths, 20))
    assert states[2][0] == 1  # the slow rank was cancelled


def test_stop_in_middle_rank_searches_again_with_seen_ids(tmp_path):
    """The consumer reaches L inside rank 1 after rank 0's IDs: rank 1 searches again with
    them as seen IDs (its own limit-L result ran past the global stop)."""
    paths = _make_blocks(str(tmp_path), dense=(2, 3))
    exp = expected(paths, 25)
    got, states = run(paths, 3, 25)
    assert key(got) == key(exp)
    assert states[1][1] == 2  # rank 1: the speculative search + the seeded one
