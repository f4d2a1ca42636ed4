"""GPU parity of the pool path (pool.hip search_pool_kernel: narrow searches).

The pool kernel hands 512-entry units to whichever wave of a CU is free and the last
units of the launch to whichever CU asks first, so records reach the host in claim
order and the host restores the reference scan order. These tests pin that order and
every record field / metric against the oracle on shapes that stress the unit space:
ragged blocks (sizes around the 512-entry unit and the 4096-entry column padding, the
32-block argument limit), tiny searches (no static units: everything dynamic), a dense
query (more matches than a workgroup's LDS record buffer — cut to 8 records so that the
test stays small: the search falls back to the segment path and the pool sits out the
next queries), host-segment growth and shrink,
and equality with an engine that never uses the pool (TSG_NO_POOL=1).

Reference anchor: tempodb/search/backend_search_block.go:184-298 (matches in page /
entry order per block), tempodb/search/backend_search_block_test.go:58-88.
"""
import os

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
CFG2 = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"},
            min_ms=10, max_ms=1000, start=T0 + 900, end=T0 + 2700)
QUERIES = [
    CFG2,
    dict(tags={"service.name": "svc-07", "http.method": "get"}),
    dict(tags={"http.method": "get", "status.code": "error"}, start=T0 + 100, end=T0 + 1500),
    dict(min_ms=500, max_ms=700),
    dict(tags={"service.name": "svc-0", "status.code": "error"}, min_ms=50),  # substring: every svc-0x value set
    dict(tags={"service.name": "no-such-service"}),
]


def request(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                           max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))


def run(engine, paths, q, limit=0):
    blocks = [engine.open_block(p) for p in paths]
    try:
        got, met = engine.search(blocks, T.Pipeline(request(q)), limit=limit)
    finally:
        for b in blocks:
            b.close()
    return [tsg_key(m) for m in got], (met.inspected_traces, met.inspected_bytes, met.inspected_blocks,
                                       met.skipped_blocks)


def oracle(paths, q, limit=0):
    exp, omet, st = O.search([O.Block(p) for p in paths], limit=limit, nthreads=1 if limit else 16, **q)
    assert st == 0
    return [match_key(m) for m in exp], (omet["traces_inspected"], omet["bytes_inspected"],
                                         omet["blocks_inspected"], omet["blocks_skipped"])


@pytest.fixture(scope="module")
def ragged(tmp_path_factory):
    """32 blocks (the one-launch argument limit), sizes around the unit / padding edges."""
    d = str(tmp_path_factory.mktemp("pool"))
    sizes = [1, 7, 511, 512, 513, 1023, 1025, 4095, 4096, 4097, 9999] + [20_000 + 3_137 * i for i in range(21)]
    paths = []
    for i, n in enumerate(sizes):
        p = os.path.join(d, "b%02d" % i)
        T.synth_search_block(p, n, seed=900 + i, profile=0, encoding=T.ENC_SNAPPY, page_size=64 << 10)
        paths.append(p)
    return paths


@pytest.fixture(scope="module")
def dyn_engine():
    """An engine that runs the claim-based pool kernel at every search size and keeps its
    dynamic tail (device-counter chunks) there (TSG_POOL_STATIC_UNITS=0, TSG_POOL_SMALL=0).
    By default a search under 32 units per workgroup (~4 M entries: every set in this file)
    runs the static-run kernel, so the default engine covers that one."""
    os.environ["TSG_POOL_SMALL"] = "0"
    os.environ["TSG_POOL_STATIC_UNITS"] = "0"
    try:
        e = T.Engine()
    finally:
        del os.environ["TSG_POOL_SMALL"]
        del os.environ["TSG_POOL_STATIC_UNITS"]
    yield e
    e.close()


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_pool_ragged_32_blocks(engine, dyn_engine, ragged, qi):
    exp = oracle(ragged, QUERIES[qi])
    assert run(engine, ragged, QUERIES[qi]) == exp
    assert run(dyn_engine, ragged, QUERIES[qi]) == exp


@pytest.mark.parametrize("limit", [1, 20, 700])
def test_pool_limit(engine, dyn_engine, ragged, limit):
    """Limit queries: every block of the wave scanned whole, each block cut to its first L
    matches on the host (the one-launch kernel's per-block caps); the consumer's distinct-id
    stop and the two-wave early exit stay in tsg_search."""
    paths = ragged[:20]  # (the oracle walks a limit query's blocks on one thread)
    for q in (CFG2, dict(tags={"service.name": "svc-07"})):
        exp = oracle(paths, q, limit)
        assert run(engine, paths, q, limit) == exp
        assert run(dyn_engine, paths, q, limit) == exp


def test_pool_tiny_searches(engine, dyn_engine, ragged):
    """Fewer units than CUs: workgroups without units (static split), or no static run at
    all and every unit claimed from the device counter (dynamic tail kept)."""
    for paths in (ragged[:1], ragged[:5], ragged[2:11]):
        for q in QUERIES[:4]:
            exp = oracle(paths, q)
            assert run(engine, paths, q) == exp
            assert run(dyn_engine, paths, q) == exp


def test_pool_dense_fallback_then_sparse(ragged):
    """More matches in a workgroup than its LDS record buffer holds (an engine whose
    buffer is cut to 8 records, TSG_POOL_REC=8; the full buffer holds 2048): the search
    reruns on the segment / look-back path and the pool sits out the next queries; every
    query of the sequence stays exact."""
    paths = ragged[11:17]
    os.environ["TSG_POOL_REC"] = "8"
    try:
        small = T.Engine()
    finally:
        del os.environ["TSG_POOL_REC"]
    try:
        dense = dict(tags={"service.name": "svc-07"})
        exp_dense, exp_sparse = oracle(paths, dense), oracle(paths, CFG2)
        got = run(small, paths, dense)
        assert len(got[0]) > 8 * 256 and got == exp_dense
        for _ in range(17):  # (past the 16 queries the pool skips after an overflow)
            assert run(small, paths, CFG2) == exp_sparse
        assert run(small, paths, dense) == exp_dense
    finally:
        small.close()


def test_pool_segment_growth_and_shrink(dyn_engine, ragged):
    """Host segments grow for a query with tens of matches per workgroup (a rerun's split
    differs from the first launch's: it can overflow again), then halve back over sparse
    queries; every query in the sequence stays exact."""
    one = dict(tags={"service.name": "svc-07"})
    exp = {"cfg2": oracle(ragged, CFG2), "one": oracle(ragged, one)}
    assert len(exp["one"][0]) > 32 * 256  # (more than a 32-record segment per workgroup on average)
    for name in ["cfg2", "one", "cfg2", "cfg2", "one", "cfg2"]:
        assert run(dyn_engine, ragged, CFG2 if name == "cfg2" else one) == exp[name]


def test_pool_matches_segment_engine(engine, ragged):
    """The pool engine and an engine without the pool return identical results."""
    os.environ["TSG_NO_POOL"] = "1"
    try:
        other = T.Engine()
    finally:
        del os.environ["TSG_NO_POOL"]
    try:
        for q in (QUERIES[0], QUERIES[2], QUERIES[3], QUERIES[5]):
            assert run(engine, ragged, q) == run(other, ragged, q)
    finally:
        other.close()


def test_aql_and_hip_launches_agree(engine, ragged):
    """The narrow kernels launched as AQL packets on libtsg's own queue (default) and through
    HIP (TSG_AQL=0) return the same records and metrics, full scans and limit queries."""
    os.environ["TSG_AQL"] = "0"
    try:
        hip = T.Engine()
        for q in QUERIES:
            for limit in (0, 20):
                assert run(engine, ragged, q, limit) == run(hip, ragged, q, limit)
    finally:
        del os.environ["TSG_AQL"]
        hip.close()
