"""Page-range parts of blocks through libtsg (tsg_block_open_pages), the GPU side of
tests/test_shard_plan.py.

Each part is searched on the device and must equal the oracle over the same part
(oracle.Block(pages=...)): records (scan positions inside the part) and metrics (a part after
page 0 counts neither the header nor the block). The parts of a size-balanced plan over 2-4
"ranks", searched in rank order (one process: a rank's search is what a rank process runs)
and merged with the frontend rule, equal the single-process search of the whole blocks —
also under a limit, where distributed_search_limit's seeded consumer is one tsg_search over
a rank's parts with the earlier ranks' IDs as seen IDs.
"""
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tempo_amd import shard
from tests.helpers import match_key, random_entries, tsg_key, write_block

pytestmark = pytest.mark.gpu

QUERY = dict(tags={"k1": "v1"}, min_ms=5)


def request(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0))


@pytest.fixture(scope="module")
def blocks(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("plan"))
    rng = random.Random(21)
    paths = []
    for b, n in enumerate([300, 1600, 120, 900]):
        ents = random_entries(rng, n)
        if b % 2:
            ents[:25] = [dict(e) for e in random_entries(random.Random(77), 25)]
            ents.sort(key=lambda e: e["id"])
        paths.append(write_block(d, f"b{b}", ents, page_size=8 << 10))
    return paths


def test_parts_match_oracle_parts(engine, blocks):
    sizes, pages = shard.block_sizes(blocks)
    assert pages[1] >= 6
    pipe = T.Pipeline(request(QUERY))
    for first, n in [(0, 2), (2, 3), (5, pages[1] - 5), (pages[1] - 1, 1), (3, 10 ** 6)]:
        part = engine.open_block(blocks[1], pages=(first, n))
        try:
            for limit in (0, 7):
                got, met = engine.search([part], pipe, limit=limit)
                exp, om, st = O.search([O.Block(blocks[1], pages=(first, min(n, 2 ** 32 - 1)))], limit=limit, **QUERY)
                assert st == 0
                assert [tsg_key(m) for m in got] == [match_key(m) for m in exp], (first, n, limit)
                assert (met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks) == (
                    om["traces_inspected"], om["bytes_inspected"], om["blocks_inspected"], om["blocks_skipped"])
        finally:
            part.close()


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("limit", [0, 30])
def test_plan_over_ranks_equals_single_process(engine, blocks, world, limit):
    sizes, pages = shard.block_sizes(blocks)
    plan = shard.plan_shards(sizes, pages, world)
    assert any(not p.whole for parts in plan for p in parts)
    pipe = T.Pipeline(request(QUERY))
    opened = [[engine.open_block(blocks[p.block], pages=p.pages()) for p in parts] for parts in plan]
    whole = [engine.open_block(p) for p in blocks]
    try:
        if limit == 0:
            wires = [engine.search_wire(bl, pipe) for bl in opened]
            got = shard.merge_wires(wires, 1 << 30, len(blocks))
            exp = shard.merge_wires([engine.search_wire(whole, pipe)], 1 << 30, len(blocks))
        else:
            # the limit protocol's outcome: ranks in order, the rank where the consumer reaches L
            # searches with the earlier ranks' distinct IDs as seen IDs, later ranks drop
            parts_resp, seen = [], None
            for bl in opened:
                r = shard.from_wire(engine.search_wire(bl, pipe, limit=limit, seen=seen))
                parts_resp.append(r)
                ids = shard._distinct_in_order(shard.concat_responses(parts_resp))
                if len(ids) >= limit:
                    break
                seen = ids if len(ids) else None
            got = shard.concat_responses(parts_resp)
            exp = shard.from_wire(engine.search_wire(whole, pipe, limit=limit))
        key = lambda r: ([bytes(x) for x in r.recs["trace_id"]], r.recs["start_ns"].tolist(),  # noqa: E731
                         (r.metrics.inspected_traces, r.metrics.inspected_bytes, r.metrics.skipped_blocks))
        assert key(got) == key(exp) and len(got) > 0
    finally:
        for bl in opened:
            for b in bl:
                b.close()
        for b in whole:
            b.close()
