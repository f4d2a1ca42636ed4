"""MatchesBlock's tag half from the device dictionary pass (pipeline.go:169-183, applied at
backend_search_block.go:219-224).

A key whose dictionary is large (> 1 MiB) and whose search-header values are verified at
open to be exactly the block's dictionary values (count + 128-bit multiset hash) has its
header test taken from the device pass ("some dictionary value contains the needle"); any
other key, or a header that differs from the entries, keeps the host scan of the header.
Both must give the oracle's results AND metrics (blocksSkipped / blocksInspected /
bytesInspected / tracesInspected): a skipped block counts its header bytes only.
"""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key, write_block

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000 * 10**9
WORDS = ["users", "orders", "items", "carts", "payments", "sessions"]


def url(rng, i):
    s = "/api/v1/" + "/".join("%s/%d" % (rng.choice(WORDS), rng.randrange(10**6)) for _ in range(10))
    return (s + "?q=%012d" % i)[:160]


def entries(seed, n, extra=None):
    rng = random.Random(seed)
    ids = sorted({bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(n)})
    out = []
    for i, tid in enumerate(ids):
        start = T0 + rng.randrange(3600 * 10**9)
        tags = {"http.url": [url(rng, i)], "service.name": ["svc-%d" % rng.randrange(5)],
                "root.service.name": ["svc-r"], "root.name": ["op-%d" % rng.randrange(3)]}
        if extra and i in extra:
            tags["http.url"] = [extra[i]]
        out.append({"id": tid, "start": start, "end": start + rng.randrange(1, 2 * 10**9), "tags": tags})
    return out


def check(engine, paths, tags, limit=0, min_ms=0):
    req = T.SearchRequest(tags=tags, min_duration_ms=min_ms)
    blocks = [engine.open_block(p) for p in paths]
    try:
        got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
    finally:
        for b in blocks:
            b.close()
    exp, omet, st = O.search([O.Block(p) for p in paths], tags=tags, limit=limit, min_ms=min_ms, nthreads=1)
    assert st == 0
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
    assert (met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks) == (
        omet["traces_inspected"], omet["bytes_inspected"], omet["blocks_inspected"], omet["blocks_skipped"])
    return got, met


@pytest.fixture(scope="module")
def wide_blocks(tmp_path_factory):
    """Three blocks of 9000 entries with ~1.4 MB of unique http.url values each (above the
    1 MiB deferral threshold); block 1 alone holds the needle 'needle-one'."""
    d = str(tmp_path_factory.mktemp("bf"))
    paths = []
    for b in range(3):
        extra = {4321: "/api/v1/needle-one/x"} if b == 1 else None
        paths.append(write_block(d, "b%d" % b, entries(70 + b, 9000, extra), page_size=256 << 10))
    return paths


def test_deferred_absent_needle_skips(engine, wide_blocks):
    got, met = check(engine, wide_blocks, {"http.url": "qqzz-not-there"})
    assert not got and met.skipped_blocks == 3 and met.inspected_blocks == 0


def test_deferred_needle_in_one_block(engine, wide_blocks):
    got, met = check(engine, wide_blocks, {"http.url": "needle-one"})
    assert len(got) == 1 and met.skipped_blocks == 2 and met.inspected_blocks == 1
    # with a narrow term beside it, a limit and a duration filter
    check(engine, wide_blocks, {"http.url": "needle-one", "service.name": "svc"}, limit=5, min_ms=1)
    check(engine, wide_blocks, {"http.url": "/orders/", "service.name": "svc-3"}, limit=20)
    check(engine, wide_blocks, {"http.url": "/orders/", "service.name": "svc-3"})


def test_header_differs_from_entries_keeps_host_filter(engine, tmp_path):
    """search-header rewritten from other entries: the header lists a value no entry has
    (the reference inspects the block and finds nothing), and lacks a value an entry has
    (the reference skips the block although an entry would match). The count/hash check at
    open fails, so the host scans the header as the reference does."""
    ents = entries(90, 9000, {100: "/api/v1/in-entries-only/1"})
    p = write_block(str(tmp_path), "hdr", ents, page_size=256 << 10)
    hdr_ents = entries(90, 9000, {100: "/api/v1/in-header-only/1"})
    with open(os.path.join(p, "search-header"), "wb") as f:
        f.write(T.fb_search_header(hdr_ents))
    got, met = check(engine, [p], {"http.url": "in-header-only"})
    assert not got and met.inspected_blocks == 1
    got, met = check(engine, [p], {"http.url": "in-entries-only"})
    assert not got and met.skipped_blocks == 1
    check(engine, [p], {"http.url": "/carts/"})


def test_cfg4_absent_needle_skipped(engine, tmp_path):
    """Config-4 profile: an absent db.statement needle skips the block on the device pass
    (24 ms of host header scan per query before)."""
    p = os.path.join(str(tmp_path), "hc")
    T.synth_search_block(p, 50_000, seed=41, profile=1)
    got, met = check(engine, [p, p], {"db.statement": "qqzz"})
    assert not got and met.skipped_blocks == 2
    got, met = check(engine, [p], {"db.statement": "where id = 77", "http.url": "/carts/"})
    assert met.inspected_blocks == 1
    check(engine, [p, p], {"db.statement": "from orders", "http.url": "qqzz"}, limit=20)


@pytest.mark.parametrize("bits", ["0", "6"])
def test_forced_hash_collisions(engine, tmp_path, wide_blocks, monkeypatch, bits):
    """the header-equals-dictionary decision must not rest on a hash. With the
    test hook TSG_VERIFY_HASH_BITS the open keeps only `bits` bits of each value's hash, so
    unequal values collide everywhere: a header that differs from the entries by one value
    must still keep the host filter, and a header equal to the dictionary must still defer —
    both with the oracle's results and metrics."""
    monkeypatch.setenv("TSG_VERIFY_HASH_BITS", bits)
    ents = entries(91, 9000, {100: "/api/v1/in-entries-only/2"})
    p = write_block(str(tmp_path), "hdr", ents, page_size=256 << 10)
    hdr_ents = entries(91, 9000, {100: "/api/v1/in-header-only/2"})
    with open(os.path.join(p, "search-header"), "wb") as f:
        f.write(T.fb_search_header(hdr_ents))
    b = engine.open_block(p)
    assert b.info()["hdr_deferred"] == 0  # one value differs: the host keeps the header test
    b.close()
    got, met = check(engine, [p], {"http.url": "in-header-only"})
    assert not got and met.inspected_blocks == 1
    got, met = check(engine, [p], {"http.url": "in-entries-only"})
    assert not got and met.skipped_blocks == 1
    for w in wide_blocks:  # header == dictionary: deferred to the device pass, collisions or not
        b = engine.open_block(w)
        assert b.info()["hdr_deferred"] == 1
        b.close()
    got, met = check(engine, wide_blocks, {"http.url": "needle-one"})
    assert len(got) == 1 and met.skipped_blocks == 2
