"""GPU parity at the shapes of BASELINE.json's five configs (the oracle checks every
match: block, scan position, trace id, start, end, DurationMs, root names, metrics).

  cfg1  one synthetic 1 M-entry block, one tag=value term        (bench.py's block 0)
  cfg2  the config-2 query (3 terms + min/max duration + time range) on that 1 M block,
        full scan and limit 20, and on three handles of it (cross-block ids, limit rule)
  cfg3  25 blocks, limit 20 against full scan: dense / medium / sparse queries cover
        the one-wave stop, the stop inside the second wave and no stop
  cfg4  high-cardinality profile (long db.statement values, ~unique http.url), 200 k
  cfg5  1 M probe ids x 200 synthetic v2 blocks (50 % present), bloom + index lookup

Reference anchor: tempodb/search/backend_search_block_test.go:58-88 (exact results and
inspected-trace counts per search).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
CFG2_TAGS = {"service.name": "svc-07", "http.method": "get", "status.code": "error"}
CFG2 = dict(tags=CFG2_TAGS, min_ms=10, max_ms=1000, start=T0 + 900, end=T0 + 2700)


def check(engine, paths, limit=0, **q):
    req = T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                          max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))
    blocks = [engine.open_block(p) for p in paths]
    try:
        got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
    finally:
        for b in blocks:
            b.close()
    exp, omet, st = O.search([O.Block(p) for p in paths], limit=limit, nthreads=1 if limit else 16, **q)
    assert st == 0
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
    assert (met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks) == (
        omet["traces_inspected"], omet["bytes_inspected"], omet["blocks_inspected"], omet["blocks_skipped"])
    return got, met


@pytest.fixture(scope="module")
def bench_block(tmp_path_factory):
    """bench.py's first block: 1 M entries, seed 0, snappy, 1 MiB pages."""
    p = os.path.join(str(tmp_path_factory.mktemp("cfg")), "r0b0")
    T.synth_search_block(p, 1_000_000, seed=0, profile=0, encoding=T.ENC_SNAPPY, page_size=1 << 20)
    return p


def test_cfg1_single_term_1m(engine, bench_block):
    got, met = check(engine, [bench_block], tags={"service.name": "svc-07"})
    assert met.inspected_traces == 1_000_000 and len(got) > 10_000


def test_cfg2_query_1m_full_and_limit20(engine, bench_block):
    got, met = check(engine, [bench_block], **CFG2)
    assert met.inspected_traces == 1_000_000 and 10 < len(got) < 1000
    got, met = check(engine, [bench_block], limit=20, **CFG2)
    assert len(got) == 20 and met.inspected_traces < 1_000_000


def test_cfg2_query_three_handles(engine, bench_block):
    """The same block three times: every id repeats across blocks (the distinct-id limit
    rule) and the records of three blocks interleave in one launch."""
    for lim in (0, 20, 700):
        check(engine, [bench_block] * 3, limit=lim, **CFG2)


@pytest.mark.parametrize("tags,min_ms", [({"status.code": ""}, 0),   # every entry with the key: dense
                                         ({"service.name": "svc-07"}, 1)])
def test_dense_limit_waves(engine, bench_block, tags, min_ms):
    """A dense query with a limit over 3 M entries (waves cut the second block): every part
    hands over at most its first L records (units keep their first L on the device, ADVICE
    r3), no rerun, and the ordered result and metrics are the oracle's; the pool path is
    still taken afterwards (a full scan right after matches the oracle too)."""
    for lim in (20, 300):
        got, met = check(engine, [bench_block] * 3, limit=lim, tags=tags, min_ms=min_ms)
        assert len(got) == lim
    req = T.SearchRequest(tags=tags, min_duration_ms=min_ms)
    blocks = [engine.open_block(bench_block) for _ in range(3)]
    try:
        got, met = engine.search(blocks, T.Pipeline(req), limit=20)
        assert met.reruns == 0
    finally:
        for b in blocks:
            b.close()
    check(engine, [bench_block], **CFG2)


@pytest.fixture(scope="module")
def cfg3_blocks(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("cfg3"))
    paths = []
    for i in range(25):
        p = os.path.join(d, "b%02d" % i)
        T.synth_search_block(p, 8000 + 97 * i, seed=300 + i, page_size=64 << 10)
        paths.append(p)
    return paths


@pytest.mark.parametrize("tags", [{"service.name": "svc-07"},                        # dense: first wave
                                  {"service.name": "svc-07", "http.method": "get"},  # medium
                                  CFG2_TAGS])                                         # sparse: no stop
def test_cfg3_limit20_vs_full(engine, cfg3_blocks, tags):
    full, fmet = check(engine, cfg3_blocks, tags=tags)
    lim, lmet = check(engine, cfg3_blocks, limit=20, tags=tags)
    assert [tsg_key(m) for m in lim] == [tsg_key(m) for m in full[:len(lim)]]
    assert lmet.inspected_traces <= fmet.inspected_traces


def test_cfg4_high_cardinality_200k(engine, tmp_path):
    p = os.path.join(str(tmp_path), "hc")
    T.synth_search_block(p, 200_000, seed=4, profile=1)
    for q in [dict(tags={"http.url": "/api/v1/users/12"}),
              dict(tags={"db.statement": "select"}),                       # every entry: dense
              dict(tags={"db.statement": "from orders", "http.url": "/carts/"}, min_ms=1),
              dict(tags={"db.statement": "where id = 77"}, start=T0 + 900, end=T0 + 2700)]:
        got, met = check(engine, [p], **q)
        assert len(got) > 0
    check(engine, [p], limit=20, tags={"db.statement": "from orders"})
    # an absent needle: MatchesBlock skips the block (blocksSkipped from the device pass)
    got, met = check(engine, [p, p], tags={"db.statement": "qqzz"})
    assert not got and met.skipped_blocks == 2
    got, met = check(engine, [p], tags={"http.url": "/carts/", "db.statement": "qqzz"}, min_ms=1)
    assert not got and met.skipped_blocks == 1


def test_cfg5_lookup_1m_probes_200_blocks(engine, tmp_path):
    paths, stored = [], []
    for b in range(200):
        p = os.path.join(str(tmp_path), "v%03d" % b)
        stored.append(T.synth_v2_block(p, 5000, seed=500 + b))
        paths.append(p)
    rng = np.random.default_rng(5)
    allstored = np.concatenate(stored)
    present = allstored[rng.integers(0, len(allstored), 500_000)]
    absent = rng.integers(0, 256, size=(500_000, 16), dtype=np.uint8)
    ids = np.concatenate([present, absent])
    rng.shuffle(ids)
    blocks = [engine.open_v2block(p) for p in paths]
    try:
        got, _ = engine.lookup(blocks, ids)
    finally:
        for b in blocks:
            b.close()
    rc, hits = O.lookup([O.V2Block(p) for p in paths], ids, nthreads=16)
    assert rc == 0
    exp = np.array(hits, dtype=np.int64).reshape(-1, 5)
    np.testing.assert_array_equal(got, exp)
    assert len(np.unique(got[:, 0])) >= 500_000  # every present probe hits its block
