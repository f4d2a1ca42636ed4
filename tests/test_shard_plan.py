"""Size-balanced shards with page-range splits (tempo_amd.shard.plan_shards), on the CPU.

SURVEY.md §8(e): blocks are assigned to ranks by bytes, in query order, and a block a cut
falls inside is split at a page boundary — the frontend's own jobs are page ranges sized by
bytes (StartPage / PagesToSearch, modules/frontend/searchsharding.go:325-367). A page range
counts the header and the block itself only when it starts at page 0, so the parts of a
block sum to the block.

Checked: the plan covers every page of every block once, in order, and balances the bytes;
over gloo ranks (world 2 and 3) on unequal blocks, the merged response of the parts equals
the single-process one — the full scan (records and metrics through the frontend merge) and
a limit query (distributed_search_limit: exactly one consumer over all blocks in order).
Without a GPU the rank's search is the oracle over its parts (oracle.Block(pages=...), the
same page-range rule); tests/test_gpu_shard_plan.py runs the parts through libtsg.
"""
import os
import random
import socket
import tempfile

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


def _check_plan(plan, sizes, pages, world, split):
    assert len(plan) == world
    seen = []  # (block, page) in rank order
    for parts in plan:
        for p in parts:
            n = pages[p.block] if p.whole else p.npages
            seen += [(p.block, p.first_page + k) for k in range(n)] if n else [(p.block, -1)]
            if not split:
                assert p.whole
    want = [(b, k) for b in range(len(sizes)) for k in range(pages[b])] + [(b, -1) for b in range(len(sizes))
                                                                           if not pages[b]]
    assert sorted(seen) == sorted(want)
    assert [x for x in seen if x[1] >= 0] == sorted(x for x in seen if x[1] >= 0)  # contiguous, in order
    total = sum(sizes)
    bpp = [s / p if p else 0 for s, p in zip(sizes, pages)]
    load = [sum(bpp[p.block] * (pages[p.block] if p.whole else p.npages) for p in parts) for parts in plan]
    slack = max(bpp) if split else max(sizes)
    assert max(load) <= total / world + slack + 1e-6


def test_plan_covers_and_balances():
    rng = random.Random(3)
    for _ in range(300):
        nb = rng.randrange(1, 9)
        pages = [rng.choice([0, 1, 2, 7, 30, 100]) for _ in range(nb)]
        sizes = [p * rng.randrange(1, 5000) for p in pages]
        for world in range(1, 7):
            for split in (True, False):
                _check_plan(shard.plan_shards(sizes, pages, world, split), sizes, pages, world, split)


def test_plan_splits_one_giant_block():
    plan = shard.plan_shards([10, 1000, 10], [1, 100, 1], 4)
    assert [len(p) for p in plan] == [2, 1, 1, 2]
    assert all(not p.whole for parts in plan for p in parts if p.block == 1)
    whole = shard.plan_shards([10, 1000, 10], [1, 100, 1], 4, split=False)
    assert [p for parts in whole for p in parts] == [shard.Part(0), shard.Part(1), shard.Part(2)]


def _make_blocks(tmpdir):
    """Unequal blocks (120 .. 1600 entries, small pages): one large block the cuts split."""
    rng = random.Random(21)
    paths = []
    for b, n in enumerate([300, 1600, 120, 500]):
        ents = random_entries(rng, n)
        if b % 2:
            ents[:25] = [dict(e) for e in random_entries(random.Random(77), 25)]  # ids shared across blocks
            ents.sort(key=lambda e: e["id"])
        paths.append(write_block(tmpdir, f"b{b}", ents, page_size=8 << 10))
    return paths


def _oracle_wire(paths, parts, limit=0, seen=None):
    blocks = [O.Block(paths[p.block], pages=p.pages()) for p in parts]
    got, met, st = O.search(blocks, limit=limit, seen=seen, **QUERY)
    assert st == 0
    traces = [T.TraceSearchMetadata(trace_id=m["id"], trace_id_len=m["id_len"],
                                    root_service_name=m["root_service"].decode(),
                                    root_trace_name=m["root_name"].decode(), start_time_unix_nano=m["start_ns"],
                                    duration_ms=m["duration_ms"]) for m in got]
    sm = T.SearchMetrics(met["traces_inspected"], met["bytes_inspected"], met["blocks_inspected"],
                         met["blocks_skipped"], block_status=[0] * len(blocks), block_errors=[None] * len(blocks))
    return shard.to_wire(shard.response_from_traces(traces, sm))


def _key(resp):
    r = resp.recs
    return ([(bytes(r["trace_id"][i]), int(r["start_ns"][i]), int(r["duration_ms"][i]), resp.name(r["root_service"][i]),
              resp.name(r["root_name"][i])) for i in range(len(r))],
            (resp.metrics.inspected_traces, resp.metrics.inspected_bytes, resp.metrics.skipped_blocks))


def _worker(rank, world, port, paths, limit, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes, pages = shard.block_sizes(paths)
        mine = shard.plan_shards(sizes, pages, world)[rank]
        if limit:
            res = shard.distributed_search_limit(lambda seen, qid: _oracle_wire(paths, mine, limit, seen),
                                                 lambda qid: None, limit)
        else:
            res = shard.distributed_search_packed(lambda: _oracle_wire(paths, mine), 1 << 30, len(paths),
                                                  columns=True)
        if rank == 0:
            np.save(os.path.join(outdir, "wire.npy"), shard.to_wire(res))
            with open(os.path.join(outdir, "parts.txt"), "w") as f:
                f.write(repr(shard.plan_shards(sizes, pages, world)))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("limit", [0, 30])
def test_split_shards_match_single_process(world, limit):
    with tempfile.TemporaryDirectory() as td:
        paths = _make_blocks(td)
        sizes, pages = shard.block_sizes(paths)
        plan = shard.plan_shards(sizes, pages, world)
        assert any(not p.whole for parts in plan for p in parts)  # the large block is split
        mp.spawn(_worker, args=(world, _free_port(), paths, limit, td), nprocs=world, join=True)
        got = shard.from_wire(np.load(os.path.join(td, "wire.npy")))
        whole = [shard.Part(b) for b in range(len(paths))]
        if limit:
            # one consumer over all blocks in order (records in order, metrics up to its stop)
            exp = shard.from_wire(_oracle_wire(paths, whole, limit))
            assert _key(got) == _key(exp) and len(got) > 0
            assert got.metrics.inspected_blocks == exp.metrics.inspected_blocks
        else:
            # the frontend merge of the parts = the frontend merge of one single-process response
            exp = shard.merge_wires([_oracle_wire(paths, whole)], 1 << 30, len(paths))
            assert _key(got) == _key(exp) and len(got) > 0
