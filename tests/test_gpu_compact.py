"""The pool kernels' compact filter column (devctx.hip `ds`: a 16-bit duration code and a
16-bit end - start span per entry, 4 B where the three 32-bit columns took 12) against the
oracle, on entries built at its edges: durations a nanosecond either side of whole
milliseconds, at and past the 16-bit code's 32767 ms, end before start (uint64 wrap, pitfall
P2), spans of 0, 65534, 65535 and more seconds and negative ones (the escape to the exact end
column). Queries put the duration bounds on those values, up to 32767 ms (the pool path) and
past it (the other paths), and the time range on the span edges.

Reference: tempodb/search/pipeline.go:30-67 (duration >= / <= in ns from whole-ms bounds;
uint32 start / end seconds overlapping [Start, End])."""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key, write_block

pytestmark = pytest.mark.gpu
MS = 1_000_000
S = 1_000_000_000
T0 = 1_700_000_000


def _entries(n=6000, seed=5):
    rng = random.Random(seed)
    durs = []
    for m in (0, 1, 10, 500, 999, 1000, 32766, 32767, 32768, 40000):
        durs += [m * MS, m * MS + 1, max(m * MS - 1, 0)]
    spans = [0, 1, 65533, 65534, 65535, 65536, 200000]
    ents = []
    ids = sorted({bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(n)})
    for i, tid in enumerate(ids):
        start = (T0 + rng.randrange(3600)) * S + rng.randrange(S)
        kind = i % 4
        if kind == 0:
            end = start + durs[rng.randrange(len(durs))]
        elif kind == 1:  # a chosen span in whole seconds (+ a sub-second part)
            end = (start // S + spans[rng.randrange(len(spans))]) * S + rng.randrange(S)
        elif kind == 2:  # end before start: the uint64 duration wraps, the span is negative
            end = start - rng.randrange(1, 10 * S) if rng.random() < 0.5 else 0
        else:
            end = start + int(rng.lognormvariate(17.7, 1.5))
        tags = {"k": ["v%d" % rng.randrange(3)], "root.service.name": ["svc"], "root.name": ["op"]}
        ents.append({"id": tid, "start": start, "end": end, "tags": tags})
    return ents


@pytest.fixture(scope="module")
def compact_blocks(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("compact"))
    return [write_block(d, "c%d" % i, _entries(seed=5 + i), page_size=64 << 10) for i in range(3)]


QUERIES = [
    dict(min_ms=1),
    dict(max_ms=1),
    dict(min_ms=1000, max_ms=1000),
    dict(min_ms=999, max_ms=1000),
    dict(min_ms=32767),
    dict(max_ms=32767),
    dict(min_ms=32766, max_ms=32767),
    dict(min_ms=32768),               # past the code: not the pool path
    dict(max_ms=40000),
    dict(start=T0 + 10, end=T0 + 20),
    dict(start=T0 + 3599, end=T0 + 4000),
    dict(start=T0 + 65534, end=T0 + 65536 + 3600),  # ends near start + 65534 .. 65536 s
    dict(start=T0 + 100000, end=T0 + 300000),
    dict(min_ms=10, max_ms=32767, start=T0 + 900, end=T0 + 2700, tags={"k": "v1"}),
]


def _req(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                           max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_compact_column_edges(engine, compact_blocks, qi):
    q = QUERIES[qi]
    exp, omet, st = O.search([O.Block(p) for p in compact_blocks], nthreads=4, **q)
    assert st == 0
    blocks = [engine.open_block(p) for p in compact_blocks]
    try:
        got, met = engine.search(blocks, T.Pipeline(_req(q)))
        got20, _ = engine.search(blocks, T.Pipeline(_req(q)), limit=20)
    finally:
        for b in blocks:
            b.close()
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
    assert (met.inspected_traces, met.inspected_blocks) == (omet["traces_inspected"], omet["blocks_inspected"])
    exp20, _, _ = O.search([O.Block(p) for p in compact_blocks], limit=20, nthreads=1, **q)
    assert [tsg_key(m) for m in got20] == [match_key(m) for m in exp20]
