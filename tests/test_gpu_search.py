"""GPU parity: libtsg search (HIP, gfx950) vs the CPU oracle on the same blocks.

Bit-exact bar: the same ordered match sequence (block, scan position, trace id,
start, end, DurationMs, root names) and the same SearchMetrics.
"""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import gen_search_data, match_key, random_entries, ref_id, tsg_key, write_block

pytestmark = pytest.mark.gpu


def both(engine, paths, tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=0):
    req = T.SearchRequest(tags=dict(tags or {}), min_duration_ms=min_ms, max_duration_ms=max_ms, start=start,
                          end=end)
    blocks = [engine.open_block(p) for p in paths]
    got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
    oblocks = [O.Block(p) for p in paths]
    exp, omet, st = O.search(oblocks, tags=tags, min_ms=min_ms, max_ms=max_ms, start=start, end=end, limit=limit)
    assert st == 0
    for b in blocks:
        b.close()
    return got, met, exp, omet


def assert_parity(got, met, exp, omet):
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
    assert met.inspected_traces == omet["traces_inspected"]
    assert met.inspected_bytes == omet["bytes_inspected"]
    assert met.inspected_blocks == omet["blocks_inspected"]
    assert met.skipped_blocks == omet["blocks_skipped"]
    assert met.block_status == omet["block_status"]


# ---- the reference's own known answers, through the GPU
@pytest.mark.parametrize("enc", [T.ENC_NONE, T.ENC_SNAPPY])
def test_backend_search_block_search(engine, tmp_path, enc):
    ents = [{"id": ref_id(i), "tags": gen_search_data(i)} for i in range(10_000)]
    p = write_block(str(tmp_path), "b", ents, enc)
    got, met, exp, omet = both(engine, [p], tags={"key20": "value_B_20"})
    assert len(got) == 1 and met.inspected_traces == 10_000
    assert_parity(got, met, exp, omet)


def test_contains_tag_table(engine, tmp_path, golden):
    g = golden["contains_tag"]
    p = write_block(str(tmp_path), "b", [{"id": ref_id(1), "tags": g["entry"]}])
    blk = engine.open_block(p)
    for c in g["cases"]:
        got, _ = engine.search([blk], T.Pipeline(T.SearchRequest(tags={c["key"]: c["value"]})))
        assert (len(got) == 1) == c["found"], c


def test_pipeline_tables(engine, tmp_path, golden):
    g = golden["pipeline"]
    for i, c in enumerate(g["tags"]):
        p = write_block(str(tmp_path), "t%d" % i, [{"id": ref_id(1), "tags": c["data"]}])
        got, _ = engine.search([engine.open_block(p)], T.Pipeline(T.SearchRequest(tags=c["req"])))
        assert (len(got) == 1) == c["match"], c["name"]
    for i, c in enumerate(g["duration"]):
        p = write_block(str(tmp_path), "d%d" % i, [{"id": ref_id(1), "start": c["start"], "end": c["end"]}])
        req = T.SearchRequest(min_duration_ms=c["min"], max_duration_ms=c["max"])
        got, _ = engine.search([engine.open_block(p)], T.Pipeline(req))
        assert (len(got) == 1) == c["match"], c["name"]
    for i, c in enumerate(g["start_end"]):
        p = write_block(str(tmp_path), "s%d" % i, [{"id": ref_id(1), "start": c["start"], "end": c["end"]}])
        got, _ = engine.search([engine.open_block(p)], T.Pipeline(T.SearchRequest(start=c["rs"], end=c["re"])))
        assert (len(got) == 1) == c["match"], c["name"]


def test_search_block_metrics(engine, tmp_path, golden):
    g = golden["search_block_metrics"]
    data = {"key1": ["value10", "value11"], "key2": ["value20", "value21"], "key3": ["value30", "value31"],
            "key4": ["value40", "value41"]}
    p = write_block(str(tmp_path), "b", [{"id": ref_id(i), "tags": data} for i in range(g["trace_count"])],
                    T.ENC_NONE)
    blk = engine.open_block(p)
    for c in g["cases"]:
        got, met = engine.search([blk], T.Pipeline(T.SearchRequest(tags=c["req"])))
        assert len(got) == c["results"]
        assert (met.inspected_blocks, met.inspected_traces, met.skipped_blocks) == (
            c["blocks_inspected"], c["traces_inspected"], c["blocks_skipped"])


# ---- randomized parity
QUERIES = [
    dict(tags={"k0": "v1"}),
    dict(tags={"k0": "v", "k1": "x"}),
    dict(tags={"k2": "v3-y", "k3": ""}),
    dict(tags={"root.service.name": "svc-1"}),
    dict(tags={"k0": "v1"}, min_ms=20, max_ms=200),
    dict(min_ms=5000),  # threshold >= 2^32 ns: exact 64-bit path
    dict(max_ms=4295),
    dict(start=1_700_000_900, end=1_700_001_800),
    dict(tags={"k1": "z", "k4": "v0"}, min_ms=1, start=1_700_000_000, end=1_700_003_000),
    dict(tags={"nokey": "v"}),
    dict(tags={"x-dbg-exhaustive": "!"}),
    dict(tags={"K0": "V1-X"}),
    dict(tags={}),
]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_blocks_parity(engine, tmp_path, seed):
    rng = random.Random(seed)
    paths = []
    for b in range(3):
        ents = random_entries(rng, rng.choice([1, 37, 700, 5000]), nkeys=5, nvals=6 + 40 * b, multi=1 + b)
        paths.append(write_block(str(tmp_path), "b%d" % b, ents, rng.choice([T.ENC_NONE, T.ENC_SNAPPY]),
                                 page_size=rng.choice([0, 4096, 65536])))
    for q in QUERIES:
        got, met, exp, omet = both(engine, paths, **q)
        assert_parity(got, met, exp, omet)


@pytest.mark.parametrize("limit", [1, 2, 5, 20, 1000])
def test_limit_parity(engine, tmp_path, limit):
    rng = random.Random(limit)
    paths = []
    shared = random_entries(rng, 50, nkeys=2, nvals=2)
    for b in range(4):
        ents = random_entries(rng, 3000, nkeys=3, nvals=3)
        # duplicate trace ids across blocks exercise the distinct-id rule
        ids = {e["id"] for e in ents}
        ents += [dict(e) for e in shared if e["id"] not in ids]
        ents.sort(key=lambda e: e["id"])
        paths.append(write_block(str(tmp_path), "b%d" % b, ents, page_size=8192))
    for q in [dict(tags={"k0": "v"}), dict(tags={"k1": "v1"}), dict(tags={"k2": "zz"})]:
        got, met, exp, omet = both(engine, paths, limit=limit, **q)
        assert_parity(got, met, exp, omet)


def test_wide_dictionaries(engine, tmp_path):
    """u16 / u32 value-set columns and bitmaps larger than the LDS budget."""
    rng = random.Random(5)
    ents = []
    for i in range(120_000):
        ents.append({"id": (i * 2654435761 % 2**64).to_bytes(8, "big") + i.to_bytes(8, "big"),
                     "start": 10**18, "end": 10**18 + i,
                     "tags": {"mid": ["m%05d" % (i % 4000)], "uniq": ["u%07d" % i],
                              "multi": ["a%d" % (i % 300), "b%d" % (i % 7)]}})
    ents.sort(key=lambda e: e["id"])
    p = write_block(str(tmp_path), "w", ents, T.ENC_SNAPPY, page_size=1 << 20)
    for q in [dict(tags={"mid": "m0001"}), dict(tags={"uniq": "u00123"}), dict(tags={"uniq": "99"}),
              dict(tags={"multi": "b3", "mid": "7"}), dict(tags={"multi": "a29"})]:
        got, met, exp, omet = both(engine, [p], **q)
        assert_parity(got, met, exp, omet)


def test_empty_and_missing_blocks(engine, tmp_path):
    p0 = write_block(str(tmp_path), "empty", [])
    ents = [{"id": ref_id(i), "tags": gen_search_data(i % 7)} for i in range(100)]
    p1 = write_block(str(tmp_path), "one", ents)
    got, met, exp, omet = both(engine, [p0, p1, p0], tags={"key3": "value"})
    assert_parity(got, met, exp, omet)
    # meta missing -> TSG_E_NOT_FOUND at open (the Go shim maps it to a no-op)
    os.remove(os.path.join(p1, "search.meta.json"))
    with pytest.raises(T.TsgError) as e:
        engine.open_block(p1)
    assert e.value.code == 1


def test_tags_and_tag_values(engine, tmp_path):
    ents = [{"id": ref_id(i), "tags": {"a": ["x%d" % (i % 3)], "b": ["y"]}} for i in range(30)]
    blk = engine.open_block(write_block(str(tmp_path), "t", ents))
    assert sorted(blk.tags()) == [b"a", b"b"]
    assert sorted(blk.tag_values(b"a")) == [b"x0", b"x1", b"x2"]
    assert blk.tag_values(b"zz") == []


def test_combine_matches_oracle(engine, tmp_path):
    rng = random.Random(11)
    shared = random_entries(rng, 40, nkeys=1, nvals=1)
    paths = []
    for b in range(3):
        ents = random_entries(rng, 500, nkeys=1, nvals=2)
        ids = {e["id"] for e in ents}
        ents += [dict(e, start=e["start"] + b) for e in shared if e["id"] not in ids]
        paths.append(write_block(str(tmp_path), "b%d" % b, ents))
    blocks = [engine.open_block(p) for p in paths]
    for lim in [0, 3, 20]:
        got, _ = engine.search_request(blocks, T.SearchRequest(tags={"k0": "v"}, limit=lim))
        exp, _, _ = O.search([O.Block(p) for p in paths], tags={"k0": "v"}, limit=lim or 20, combine=lim or 20)
        assert [(m.trace_id, m.start_time_unix_nano, m.duration_ms, m.root_service_name.encode())
                for m in got] == [(e["id"], e["start_ns"], e["duration_ms"], e["root_service"]) for e in exp]


def test_synthetic_block_full_scan(engine, tmp_path):
    p = os.path.join(str(tmp_path), "syn")
    T.synth_search_block(p, 60_000, seed=3)
    q = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"}, min_ms=10,
             max_ms=1000, start=1_700_000_900, end=1_700_002_700)
    for qq in [q, dict(tags={"service.name": "svc-07"}), dict(tags={"name": "span-001"}),
               dict(tags={"http.url": "/users/12"})]:
        got, met, exp, omet = both(engine, [p], **qq)
        assert_parity(got, met, exp, omet)


def test_match_everything_regrows_result_buffer(tmp_path):
    """An unfiltered query on a fresh context: the first result buffer (2^16
    records) overflows and the emit pass re-runs into a larger one. Every entry
    matches, in scan order."""
    p = os.path.join(str(tmp_path), "big")
    n = (1 << 16) * 2 + 777
    T.synth_search_block(p, n, seed=11)
    engine = T.Engine(devices=[0])
    b = engine.open_block(p)
    try:
        got, met = engine.search([b], T.Pipeline(T.SearchRequest()))
        assert len(got) == n and met.inspected_traces == n
        assert all(m.entry_idx == i for i, m in enumerate(got))
        n2, met2 = engine.search_raw([b], T.Pipeline(T.SearchRequest(tags={"service.name": "svc-07"})))
        got3, _ = engine.search([b], T.Pipeline(T.SearchRequest(tags={"service.name": "svc-07"})))
        assert n2 == len(got3) and 0 < n2 < n
        exp, omet, _ = O.search([O.Block(p)], tags={"service.name": "svc-07"})
        assert [tsg_key(m) for m in got3] == [match_key(m) for m in exp]
    finally:
        b.close()
        engine.close()


def test_timing_flags(engine, tmp_path):
    p = os.path.join(str(tmp_path), "syn")
    T.synth_search_block(p, 50_000, seed=5)
    b = engine.open_block(p)
    try:
        pipe = T.Pipeline(T.SearchRequest(tags={"service.name": "svc-07"}, min_duration_ms=10))
        _, m0 = engine.search_raw([b], pipe)
        assert m0.scan_kernel_ns == 0 and m0.kernel_ns == 0
        _, m1 = engine.search_raw([b], pipe, flags=T.SEARCH_TIME_SCAN)
        assert m1.scan_kernel_ns > 0 and m1.kernel_ns == 0
        _, m2 = engine.search_raw([b], pipe, flags=T.SEARCH_TIME_ALL)
        assert m2.kernel_ns >= m2.scan_kernel_ns > 0
        assert m1.scan_bytes == m2.scan_bytes > 0
        engine.kernel_times()  # drain
        for _ in range(3):
            _, m3 = engine.search_raw([b], pipe, flags=T.SEARCH_TIME_DEFER)
            assert m3.scan_kernel_ns == 0
        ts = engine.kernel_times()
        assert len(ts) == 3 and all(t > 0 for t in ts)
        assert engine.kernel_times() == []
    finally:
        b.close()


def test_result_modes_switch_with_match_density(tmp_path):
    """Segment mode (per-tile record segments) grows its segments when a tile
    overflows, hands dense queries to look-back mode and returns to segments when
    results are sparse again: the same ordered matches as the oracle throughout."""
    p = os.path.join(str(tmp_path), "dens")
    T.synth_search_block(p, 300_000, seed=21)
    engine = T.Engine(devices=[0])
    b = engine.open_block(p)
    ob = O.Block(p)
    try:
        for tags in [{"service.name": "svc-07"},   # ~40 per tile: 16-record segments overflow
                     {"span.kind": "s"},           # dense: look-back mode
                     {"service.name": "svc-07"},
                     {"service.name": "svc-07", "http.method": "get", "status.code": "error"},  # sparse
                     {"service.name": "svc-1"},
                     {"http.method": "post"}]:
            got, _ = engine.search([b], T.Pipeline(T.SearchRequest(tags=tags)))
            exp, _, _ = O.search([ob], tags=tags)
            assert [tsg_key(m) for m in got] == [match_key(m) for m in exp], tags
            for lim in (3, 20):
                got, _ = engine.search([b], T.Pipeline(T.SearchRequest(tags=tags)), limit=lim)
                exp, _, _ = O.search([ob], tags=tags, limit=lim)
                assert [tsg_key(m) for m in got] == [match_key(m) for m in exp], (tags, lim)
    finally:
        b.close()
        engine.close()


def test_many_blocks_general_path(engine, tmp_path):
    """More blocks than the one-launch path's kernel arguments carry (32): tsg_search
    splits them into chunks of 32 blocks per launch (TSG_CHUNK_BLOCKS=0: one descriptor-
    path launch for all, run by tools/gpu_round.sh), with the same results."""
    rng = random.Random(42)
    paths = [write_block(str(tmp_path), f"b{i}", random_entries(rng, 150)) for i in range(40)]
    for q in [dict(tags={"k1": "v1"}), dict(tags={"k2": "v3-x", "root.service.name": "svc"}, min_ms=1),
              dict(min_ms=3, max_ms=5000)]:
        got, met, exp, omet = both(engine, paths, **q)
        assert_parity(got, met, exp, omet)
    got, met, exp, omet = both(engine, paths, tags={"k1": "v"}, limit=7)
    assert_parity(got, met, exp, omet)


def test_high_cardinality_config4(engine, tmp_path):
    """BASELINE config 4 shape: ~unique http.url and long db.statement values
    (substring terms over large dictionaries: the prep-kernel path)."""
    p = os.path.join(str(tmp_path), "hc")
    T.synth_search_block(p, 20_000, seed=4, profile=1)
    for q in [dict(tags={"http.url": "/api/v1/users/12"}),
              dict(tags={"db.statement": "select"}),
              dict(tags={"http.url": "/api/v1/users/12", "db.statement": "from orders"}, min_ms=1),
              dict(tags={"db.statement": "where id = 77"}, start=1_700_000_900, end=1_700_002_700)]:
        got, met, exp, omet = both(engine, [p], **q)
        assert_parity(got, met, exp, omet)
        assert len(exp) > 0


@pytest.mark.parametrize("limit", [1, 20, 300, 5000])
def test_limit_early_exit_waves(engine, tmp_path, limit):
    """limit > 0 over many blocks: the leading blocks are searched first and the rest
    only when the consumer has not stopped inside them (tsg_search's two waves). Dense
    queries stop in the first wave, sparse ones need the second; both must equal the
    oracle's single sequential pass, metrics included."""
    rng = random.Random(100 + limit)
    paths = []
    for b in range(10):
        ents = random_entries(rng, 2000 + 300 * b, nkeys=3, nvals=4)
        paths.append(write_block(str(tmp_path), "w%d" % b, ents, page_size=16384))
    for q in [dict(tags={"k0": "v"}),            # dense: stops in block 0
              dict(tags={"k1": "v1-x"}),         # medium
              dict(tags={"k2": "v3-z", "k0": "v2"}, min_ms=50)]:  # sparse: all blocks
        got, met, exp, omet = both(engine, paths, limit=limit, **q)
        assert_parity(got, met, exp, omet)


def test_cancel(engine, tmp_path):
    """tsg_cancel (the Go shim's ctx.Done()): cooperative, checked before every device
    chunk (32 blocks per launch) and between waves. A search cancelled before it starts
    always returns TSG_E_CANCELLED; cancelled from another thread while it runs, it
    returns TSG_E_CANCELLED or its complete, correct result (the reference's AddResult
    returns quit on ctx.Done() and the consumer reads nothing more, results.go:38-52)."""
    import threading
    import time
    rng = random.Random(77)
    paths = [write_block(str(tmp_path), "c%d" % i, random_entries(rng, 1500, nkeys=2, nvals=3)) for i in range(70)]
    blocks = [engine.open_block(p) for p in paths]
    try:
        pipe = T.Pipeline(T.SearchRequest(tags={"k0": "v"}))
        full, fmet = engine.search(blocks, pipe)
        exp, _, _ = O.search([O.Block(p) for p in paths], tags={"k0": "v"})
        assert [tsg_key(m) for m in full] == [match_key(m) for m in exp]
        engine.cancel(1001)
        with pytest.raises(T.TsgError) as e:
            engine.search(blocks, pipe, query_id=1001)
        assert e.value.code == T.TSG_E_CANCELLED
        got, _ = engine.search(blocks, pipe, query_id=1001)  # the id was consumed by that search
        assert [tsg_key(m) for m in got] == [tsg_key(m) for m in full]
        engine.cancel(5)
        got, _ = engine.search(blocks, pipe, query_id=6)  # another id's cancel: no effect
        assert [tsg_key(m) for m in got] == [tsg_key(m) for m in full]
        outcomes = []
        for i in range(12):
            qid = 2000 + i
            go = threading.Event()

            def canceller(q=qid, d=i * 40e-6):
                go.wait()
                time.sleep(d)
                engine.cancel(q)

            th = threading.Thread(target=canceller)
            th.start()
            go.set()
            try:
                got, _ = engine.search(blocks, pipe, query_id=qid, limit=0)
                assert [tsg_key(m) for m in got] == [tsg_key(m) for m in full]
                outcomes.append("done")
            except T.TsgError as e:
                assert e.code == T.TSG_E_CANCELLED
                outcomes.append("cancelled")
            th.join()
            # a cancel that came after its search returned is dropped: the id can
            # be reused at once
            again, _ = engine.search(blocks, pipe, query_id=qid)
            assert [tsg_key(m) for m in again] == [tsg_key(m) for m in full]
        print("cancel outcomes:", outcomes)
        # the race in its plain form: search, then a late cancel, then the id again
        engine.search(blocks[:1], pipe, query_id=4242)
        engine.cancel(4242)
        got, _ = engine.search(blocks, pipe, query_id=4242)
        assert [tsg_key(m) for m in got] == [tsg_key(m) for m in full]
    finally:
        for b in blocks:
            b.close()


def test_block_clone(engine, tmp_path):
    """tsg_block_clone: a second resident copy searches exactly like the original, and
    outlives it."""
    rng = random.Random(91)
    paths = [write_block(str(tmp_path), "k%d" % i, random_entries(rng, 900, nkeys=3, nvals=5, multi=2))
             for i in range(2)]
    wal = os.path.join(str(tmp_path), T.wal_filename())
    T.write_wal_search(wal, random_entries(rng, 300, nkeys=2, nvals=3))
    orig = [engine.open_block(p) for p in paths] + [engine.open_wal_block(wal)]
    pipe = T.Pipeline(T.SearchRequest(tags={"k1": "v"}, min_duration_ms=2))
    exp, emet = engine.search(orig, pipe)
    clones = [b.clone(engine) for b in orig]
    assert [c.info()["entries"] for c in clones] == [b.info()["entries"] for b in orig]
    for b in orig:
        b.close()
    got, gmet = engine.search(clones, pipe)
    assert [tsg_key(m) for m in got] == [tsg_key(m) for m in exp]
    assert (gmet.inspected_traces, gmet.inspected_bytes) == (emet.inspected_traces, emet.inspected_bytes)
    for c in clones:
        c.close()


def test_header_min_dur_quirk_skips_block(engine, tmp_path):
    """Pitfall P1 through a full search: SearchBlockHeaderMutable.AddEntry overwrites a zero
    MinDur with the next entry's duration (pkg/tempofb/SearchBlockHeader_util.go:37-43), so
    the stored MinDur (5 s) exceeds the block's true minimum (0). MatchesBlock compares the
    stored value with MaxDurationMs (tempodb/search/pipeline.go:53-56): a MaxDuration query
    skips the whole block although its zero-duration entry matches; the block without the
    quirk is inspected. Both on the on-disk header, as the reference."""
    t0 = 1_700_000_000 * 10**9
    quirk = [{"id": ref_id(1), "start": t0, "end": t0, "tags": {"k": ["a"]}},            # dur 0 (AddEntry first)
             {"id": ref_id(2), "start": t0, "end": t0 + 5 * 10**9, "tags": {"k": ["a"]}},  # 5 s: MinDur := 5 s
             {"id": ref_id(3), "start": t0, "end": t0 + 6 * 10**9, "tags": {"k": ["a"]}}]
    plain = [{"id": ref_id(4), "start": t0, "end": t0 + 10**6, "tags": {"k": ["a"]}},     # 1 ms
             {"id": ref_id(5), "start": t0, "end": t0 + 5 * 10**9, "tags": {"k": ["a"]}}]
    pq = write_block(str(tmp_path), "quirk", quirk)
    pp = write_block(str(tmp_path), "plain", plain)
    assert engine.open_block(pq).info()["min_dur_ns"] == 5 * 10**9  # the stored (overwritten) MinDur
    got, met, exp, omet = both(engine, [pq, pp], tags={"k": "a"}, max_ms=1000)
    assert met.skipped_blocks == 1 and met.inspected_blocks == 1
    assert [(m.block_idx, m.trace_id) for m in got] == [(1, ref_id(4))]  # ref_id(1) (0 ns) is not found
    assert_parity(got, met, exp, omet)
    # without MaxDuration the quirk block is searched and its zero-duration entry matches
    got, met, exp, omet = both(engine, [pq, pp], tags={"k": "a"})
    assert met.skipped_blocks == 0 and ref_id(1) in [m.trace_id for m in got]
    assert_parity(got, met, exp, omet)


def test_search_raw_tuple_identity_cache(engine, tmp_path):
    """search_raw's identity fast path for tuple block lists: the same tuple gives the
    same count as a list of the same blocks, and closing any block invalidates the entry
    (the call then fails on the closed handle instead of using it)."""
    p = os.path.join(str(tmp_path), "syn")
    T.synth_search_block(p, 20_000, seed=9)
    b = engine.open_block(p)
    c = b.clone(engine)
    pipe = T.Pipeline(T.SearchRequest(tags={"service.name": "svc-07"}))
    try:
        blocks = (b, c)
        n_list, _ = engine.search_raw([b, c], pipe)
        for _ in range(3):
            n_tup, _ = engine.search_raw(blocks, pipe, metrics=False)
            assert n_tup == n_list > 0
        n_lim, _ = engine.search_raw(blocks, pipe, limit=5)
        assert 0 < n_lim <= n_list
        c.close()
        with pytest.raises(Exception):
            engine.search_raw(blocks, pipe)
    finally:
        c.close()
        b.close()


def test_concurrent_opens_match_oracle(engine, tmp_path):
    """Blocks opened from several threads at once (the loader then splits the CPUs between
    the decodes, and the uploads prepare their arrays outside the device lock): every block's
    columns, dictionaries and names come out as the oracle reads them."""
    from concurrent.futures import ThreadPoolExecutor
    specs = [(40_000, 21, 0, T.ENC_SNAPPY), (20_000, 22, 1, T.ENC_SNAPPY), (30_000, 23, 0, T.ENC_NONE),
             (40_000, 24, 0, T.ENC_SNAPPY)]
    paths = []
    for i, (n, seed, prof, enc) in enumerate(specs):
        p = os.path.join(str(tmp_path), f"c{i}")
        T.synth_search_block(p, n, seed=seed, profile=prof, encoding=enc, page_size=64 * 1024)
        paths.append(p)
    with ThreadPoolExecutor(len(paths)) as ex:
        blocks = list(ex.map(engine.open_block, paths))
    try:
        oblocks = [O.Block(p) for p in paths]
        for tags, mn, mx in [({"service.name": "svc-07"}, 10, 1000), ({"http.method": "get", "status.code": "1"}, 0, 0),
                             ({"name": "span-0042"}, 0, 0)]:
            req = T.SearchRequest(tags=tags, min_duration_ms=mn, max_duration_ms=mx)
            got, met = engine.search(blocks, T.Pipeline(req))
            exp, omet, st = O.search(oblocks, tags=tags, min_ms=mn, max_ms=mx)
            assert st == 0 and len(exp) > 0
            assert_parity(got, met, exp, omet)
    finally:
        for b in blocks:
            b.close()
