"""GPU parity for live-trace search (instance.searchLiveTraces, modules/ingester/
instance_search.go:83-130) and Tags / TagValues (backend_search_block.go:145-181,
streaming_search_block.go:97-116, instance_search.go:187-273): libtsg's live block (one row
per searchData segment, matched by the HIP search kernels, combined per trace on the host)
vs the oracle's restatement, bit-exact: ordered results, every result field, the metrics,
limits, mixed-case keys (pitfall P3), empty ids, live + WAL + backend blocks in one search;
tags and tag values of every block kind and the instance aggregation with its size limit."""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import random_entries, ref_id
from tests.test_gpu_search import assert_parity

pytestmark = pytest.mark.gpu


def seg(tid, tags, start=0, end=0):
    return T.fb_search_entry({"id": tid, "start": start, "end": end, "tags": tags})


def both(engine, traces, tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=0, extra=(), extra_o=()):
    req = T.SearchRequest(tags=dict(tags or {}), min_duration_ms=min_ms, max_duration_ms=max_ms, start=start,
                          end=end)
    lb = engine.open_live_traces(traces)
    got, met = engine.search([lb] + list(extra), T.Pipeline(req), limit=limit)
    exp, omet, st = O.search([O.LiveBlock(traces)] + list(extra_o), tags=tags, min_ms=min_ms, max_ms=max_ms,
                             start=start, end=end, limit=limit)
    assert st == 0
    lb.close()
    return got, met, exp, omet


def random_live(rng, ntraces, t0=1_700_000_000 * 10**9, mixed_case=False):
    """Live traces: 0-4 segments each (segments of one trace usually share its id), tags from a
    small vocabulary so segments of a trace agree and disagree, zero / wrapped durations."""
    traces = []
    for t in range(ntraces):
        tid = rng.getrandbits(128).to_bytes(16, "big") if rng.random() > 0.02 else b""
        segs = []
        for _ in range(rng.choice([0, 1, 1, 1, 2, 2, 3, 4])):
            tags = {}
            for k in range(5):
                if rng.random() < 0.7:
                    key = "k%d" % k
                    if mixed_case and rng.random() < 0.3:
                        key = key.upper()
                    tags[key] = sorted({"v%d%s" % (rng.randrange(4), "xyz"[rng.randrange(3)])
                                        for _ in range(1 + rng.randrange(2))})
            if rng.random() < 0.6:
                tags["root.service.name"] = ["svc-%d" % rng.randrange(3)]
            if rng.random() < 0.6:
                tags["root.name"] = ["op-%d" % rng.randrange(5)]
            start = t0 + rng.randrange(3600 * 10**9)
            end = start + int(rng.lognormvariate(17.7, 1.5))
            if rng.random() < 0.03:
                end = 0
            sid = tid if rng.random() > 0.05 else rng.getrandbits(128).to_bytes(16, "big")
            segs.append(seg(sid, tags, start, end))
        traces.append(segs)
    return traces


def test_instance_search_live_stage(engine, golden):
    """TestInstanceSearch's live stage (instance_search_test.go:41-97) through the GPU."""
    g = golden["instance_search_live"]["search"]
    k, v = g["tag"]
    rng = random.Random(1)
    traces = []
    for j in range(g["num_traces"]):
        tid = bytes(rng.getrandbits(8) for _ in range(16))
        traces.append([seg(tid, {k: [v]})] if j % g["annotated_every"] == 0 else [])
    got, met, exp, omet = both(engine, traces, tags={k: v})
    assert len(got) == g["expected_results"] and met.inspected_traces == g["num_traces"]
    assert_parity(got, met, exp, omet)
    res, _ = engine.search_request([engine.open_live_traces(traces)], T.SearchRequest(tags={k: v}))
    assert len(res) == g["expected_results"]


def test_instance_search_metrics_live_stage(engine, golden):
    """TestInstanceSearchMetrics (:331-371): exhaustive search inspects every live trace and
    every segment byte."""
    g = golden["instance_search_live"]["metrics"]
    k, v = g["tag"]
    rng = random.Random(2)
    traces = [[seg(bytes(rng.getrandbits(8) for _ in range(16)), {k: [v]})] for _ in range(g["num_traces"])]
    got, met, exp, omet = both(engine, traces, tags={"x-dbg-exhaustive": "!"})
    assert got == [] and met.inspected_traces == g["expected_traces_inspected"]
    assert met.inspected_bytes == sum(len(t[0]) for t in traces)
    assert_parity(got, met, exp, omet)


def test_combine_fields(engine):
    tid = ref_id(7)
    traces = [[seg(tid, {"k": ["a"]}, 1_000_000_000, 1_005_000_000),
               seg(tid, {"k": ["zzz"], "root.service.name": ["nope"]}, 1, 2),
               seg(tid, {"k": ["a"], "root.service.name": ["svc"], "root.name": ["op"]}, 900_000_000, 910_000_000)],
              [seg(b"", {"k": ["a"]}), seg(ref_id(9), {"k": ["a"], "root.name": ["x"]})]]
    got, met, exp, omet = both(engine, traces, tags={"k": "a"})
    assert [(m.entry_idx, m.duration_ms, m.root_service_name) for m in got] == [(0, 10, "svc"), (1, 0, "")]
    assert got[1].trace_id == ref_id(9)
    assert_parity(got, met, exp, omet)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_random_live_parity(engine, seed):
    rng = random.Random(100 + seed)
    traces = random_live(rng, 3000, mixed_case=seed % 2 == 1)
    queries = [dict(tags={"k1": "v1"}), dict(tags={"k0": "x", "k2": "v"}), dict(tags={"K3": "v"}),
               dict(tags={"k4": ""}, min_ms=5, max_ms=500), dict(tags={}, start=1_700_000_900, end=1_700_002_700),
               dict(tags={"root.service.name": "svc-1"}), dict(tags={"nokey": "a"})]
    for q in queries:
        for limit in (0, 1, 7, 50):
            got, met, exp, omet = both(engine, traces, limit=limit, **q)
            assert_parity(got, met, exp, omet)


def test_live_wal_backend_one_search(engine, tmp_path):
    """instance.Search's three sources in one ordered sequence: live traces, a WAL block, a
    backend block (caller order), with limits cutting inside each of them."""
    rng = random.Random(5)
    traces = random_live(rng, 400)
    wp = os.path.join(str(tmp_path), T.wal_filename())
    T.write_wal_search(wp, random_entries(rng, 300, nkeys=5, nvals=4))
    bp = os.path.join(str(tmp_path), "b")
    T.write_search_block(bp, random_entries(rng, 2000, nkeys=5, nvals=4))
    wb, bb = engine.open_wal_block(wp), engine.open_block(bp)
    for limit in (0, 3, 40, 200, 1000):
        got, met, exp, omet = both(engine, traces, tags={"k1": "v1"}, limit=limit, extra=[wb, bb],
                                   extra_o=[O.Block(wp, wal=True), O.Block(bp)])
        assert_parity(got, met, exp, omet)


def test_empty_and_segmentless(engine):
    for traces in ([], [[]], [[], [], []]):
        got, met, exp, omet = both(engine, traces, tags={"k": "a"})
        assert got == [] and met.inspected_traces == len(traces)
        assert_parity(got, met, exp, omet)
    with pytest.raises(T.TsgError) as e:
        engine.open_live_traces([[b"\x01\x00"]])
    assert e.value.code == T.TSG_E_CORRUPT


def test_live_block_info(engine):
    traces = random_live(random.Random(3), 50)
    lb = engine.open_live_traces(traces)
    info = lb.info()
    assert info["live"] == 1 and info["traces"] == 50 and info["entries"] == sum(len(t) for t in traces)
    assert info["fb_bytes"] == sum(len(s) for t in traces for s in t)
    lb.close()


# ---- Tags / TagValues ------------------------------------------------------------------
def _oracle_ok(res):
    st, v = res
    assert st == 0
    return v


def test_tags_every_block_kind(engine, tmp_path):
    rng = random.Random(11)
    ents = random_entries(rng, 500, nkeys=6, nvals=6)
    bp = os.path.join(str(tmp_path), "b")
    T.write_search_block(bp, ents)
    wp = os.path.join(str(tmp_path), T.wal_filename())
    T.write_wal_search(wp, ents[:200] + ents[:50])
    traces = random_live(rng, 300, mixed_case=True)
    blocks = [engine.open_block(bp), engine.open_wal_block(wp), engine.open_live_traces(traces)]
    oblocks = [O.Block(bp), O.Block(wp, wal=True), O.LiveBlock(traces)]
    keys = set()
    for b, ob in zip(blocks, oblocks):
        got = b.tags()
        assert got == _oracle_ok(O.block_tags(ob))
        keys.update(got)
        for k in sorted(keys) + [b"nokey", b"K1", b"root.name"]:
            assert b.tag_values(k) == _oracle_ok(O.block_tag_values(ob, k)), (b, k)
    # the instance aggregation: live first, then the rest; the size limit after each stage
    assert engine.search_tags(blocks) == _oracle_ok(O.search_tags(oblocks))
    for k in [b"k0", b"k1", b"K2", b"root.service.name", b"root.name"]:
        full = engine.search_tag_values(blocks, k)
        assert full == _oracle_ok(O.search_tag_values(oblocks, k))
        size = sum(len(v) for v in full)
        for mb in (-1, 0, 1, size // 2, size, size + 1):
            assert engine.search_tag_values(blocks, k, mb) == _oracle_ok(O.search_tag_values(oblocks, k, mb)), (k, mb)
    for b in blocks:
        b.close()
