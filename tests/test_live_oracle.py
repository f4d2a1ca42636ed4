"""Live traces (instance.searchLiveTraces, modules/ingester/instance_search.go:83-130) and
SearchTags / SearchTagValues (backend_search_block.go:145-181, streaming_search_block.go:97-116,
instance_search.go:187-273) in the CPU oracle, pinned to the reference's own tests where they
hold answers (TestInstanceSearch / TestInstanceSearchMetrics' live-trace stage, parsed into
tests/golden/known_answers.json) and to CombineSearchResults' rules. CPU only; the engine side
is tests/test_gpu_live.py."""
import os
import random

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import ref_id


def seg(tid, tags, start=0, end=0):
    """SearchEntryMutable{TraceID, tags, start, end}.ToBytes (the distributor's searchData)."""
    return O.entry_to_bytes({"id": tid, "start": start, "end": end, "tags": tags})


def test_instance_search_live_stage(golden):
    """TestInstanceSearch (instance_search_test.go:41-97) before any cut: 500 live traces,
    every 100th with search data {foo: bar}, the rest with none -> 5 results, and every
    live trace counts as inspected."""
    g = golden["instance_search_live"]["search"]
    k, v = g["tag"]
    rng = random.Random(1)
    traces, ids = [], []
    for j in range(g["num_traces"]):
        tid = bytes(rng.getrandbits(8) for _ in range(16))
        if j % g["annotated_every"] == 0:
            traces.append([seg(tid, {k: [v]})])
            ids.append(tid)
        else:
            traces.append([])
    lb = O.LiveBlock(traces)
    m, met, st = O.search([lb], tags={k: v})
    assert st == 0 and len(m) == g["expected_results"]
    assert sorted(x["id"] for x in m) == sorted(ids)
    assert met["traces_inspected"] == g["num_traces"] and met["blocks_inspected"] == 0
    # instance.Search's consumer (limit 20 default) keeps all 5, sorted by start descending
    c, _, _ = O.search([lb], tags={k: v}, combine=20)
    assert len(c) == g["expected_results"]


def test_instance_search_metrics_live_stage(golden):
    """TestInstanceSearchMetrics (:331-371): an exhaustive search of 500 live traces inspects
    every trace and the sum of the segments' lengths."""
    g = golden["instance_search_live"]["metrics"]
    k, v = g["tag"]
    rng = random.Random(2)
    traces, nbytes = [], 0
    for _ in range(g["num_traces"]):
        s = seg(bytes(rng.getrandbits(8) for _ in range(16)), {k: [v]})
        nbytes += len(s)
        traces.append([s])
    m, met, st = O.search([O.LiveBlock(traces)], tags={"x-dbg-exhaustive": "!"})
    assert st == 0 and m == []
    assert met["traces_inspected"] == g["expected_traces_inspected"] and met["bytes_inspected"] == nbytes


def test_segments_match_alone_and_combine():
    """Each segment is matched on its own; a trace's matching segments fold with
    CombineSearchResults: first non-empty names, earliest start, longest DurationMs
    (tempodb/search/util.go:40-62). bytesInspected counts every segment, matching or not."""
    tid = ref_id(7)
    s1 = seg(tid, {"k": ["a"]}, start=1_000_000_000, end=1_005_000_000)          # 5 ms, no names
    s2 = seg(tid, {"k": ["zzz"], "root.service.name": ["nope"]}, start=1, end=2)  # does not match
    s3 = seg(tid, {"k": ["a"], "root.service.name": ["svc"], "root.name": ["op"]},
             start=900_000_000, end=910_000_000)                                  # 10 ms
    lb = O.LiveBlock([[s1, s2, s3]])
    m, met, st = O.search([lb], tags={"k": "a"})
    assert st == 0 and len(m) == 1
    r = m[0]
    assert (r["id"], r["start_ns"], r["duration_ms"], r["root_service"], r["root_name"], r["entry_idx"]) == \
        (tid, 900_000_000, 10, b"svc", b"op", 0)
    assert met["traces_inspected"] == 1 and met["bytes_inspected"] == len(s1) + len(s2) + len(s3)
    # a segment-level trace filter: only s1 is >= 5 ms and <= 6 ms -> its own fields
    m, _, _ = O.search([lb], tags={"k": "a"}, min_ms=5, max_ms=6)
    assert len(m) == 1 and (m[0]["start_ns"], m[0]["duration_ms"], m[0]["root_service"]) == (1_000_000_000, 5, b"")


def test_empty_trace_id_takes_the_next_segments():
    """existing.TraceID == "" (an all-zero / empty id) takes the incoming one."""
    real = ref_id(9)
    lb = O.LiveBlock([[seg(b"", {"k": ["a"]}), seg(real, {"k": ["a"]})]])
    m, _, _ = O.search([lb], tags={"k": "a"})
    assert len(m) == 1 and m[0]["id"] == real and m[0]["id_len"] == 16


def test_limit_stops_after_the_trace():
    """The consumer closes on the L-th distinct id: tracesInspected / bytesInspected run up to
    and including that trace (deterministic refinement of the racy reference)."""
    traces, lens = [], []
    for i in range(10):
        segs = [seg(ref_id(i), {"k": ["a" if i % 2 == 0 else "b"]})] * (1 + i % 3)
        traces.append(segs)
        lens.append(sum(len(s) for s in segs))
    lb = O.LiveBlock(traces)
    m, met, _ = O.search([lb], tags={"k": "a"}, limit=3)
    assert [x["entry_idx"] for x in m] == [0, 2, 4]
    assert met["traces_inspected"] == 5 and met["bytes_inspected"] == sum(lens[:5])


def test_live_then_blocks_in_one_search(tmp_path):
    """Live traces, then a backend block: one ordered sequence (block order = caller order)."""
    ents = [{"id": ref_id(100 + i), "start": 5, "end": 6, "tags": {"k": ["a"]}} for i in range(4)]
    p = os.path.join(str(tmp_path), "b")
    T.write_search_block(p, ents)
    lb = O.LiveBlock([[seg(ref_id(1), {"k": ["a"]})], [seg(ref_id(2), {"k": ["c"]})]])
    m, met, _ = O.search([lb, O.Block(p)], tags={"k": "a"})
    assert [(x["block_idx"], x["entry_idx"]) for x in m] == [(0, 0), (1, 0), (1, 1), (1, 2), (1, 3)]
    assert met["blocks_inspected"] == 1 and met["traces_inspected"] == 2 + 4


def test_mixed_case_keys_live():
    """Pitfall P3 on live segments: keys sorted by original case then lowercased can leave
    the vector ascending; FindTag's binary search then misses "a" (Search and TagValues),
    while Tags lists every key."""
    s = seg(ref_id(1), {"B": ["x"], "a": ["y"]})
    lb = O.LiveBlock([[s]])
    assert len(O.search([lb], tags={"a": "y"})[0]) == 0
    assert len(O.search([lb], tags={"b": "x"})[0]) == 1
    assert O.block_tags(lb) == (0, [b"a", b"b"])
    assert O.block_tag_values(lb, b"a") == (0, [])
    assert O.block_tag_values(lb, b"b") == (0, [b"x"])


def test_tags_backend_wal_live(tmp_path):
    ents = [{"id": ref_id(i), "tags": {"a": ["x%d" % (i % 3)], "b": ["y"]}} for i in range(6)]
    bp = os.path.join(str(tmp_path), "b")
    T.write_search_block(bp, ents)
    wp = os.path.join(str(tmp_path), T.wal_filename())
    T.write_wal_search(wp, ents)
    lb = O.LiveBlock([[seg(ref_id(50), {"c": ["z1", "z2"], "a": ["x9"]})]])
    for b in (O.Block(bp), O.Block(wp, wal=True)):
        assert O.block_tags(b) == (0, [b"a", b"b"])
        assert O.block_tag_values(b, b"a") == (0, [b"x0", b"x1", b"x2"])
        assert O.block_tag_values(b, b"zz") == (0, [])
    assert O.block_tags(lb) == (0, [b"a", b"c"])
    blocks = [O.Block(bp), O.Block(wp, wal=True), lb]
    assert O.search_tags(blocks) == (0, [b"a", b"b", b"c"])
    assert O.search_tag_values(blocks, b"a") == (0, [b"x0", b"x1", b"x2", b"x9"])
    # util.MapSizeWithinLimit: sum of the distinct values' lengths must stay below the limit
    assert O.search_tag_values(blocks, b"a", max_bytes=8) == (0, [])  # 8 bytes after all blocks: not < 8
    assert O.search_tag_values(blocks, b"a", max_bytes=9)[1] == [b"x0", b"x1", b"x2", b"x9"]
    assert O.search_tag_values(blocks, b"a", max_bytes=3)[1] == []  # 2 bytes after live, 8 after all
    assert O.search_tag_values(blocks, b"a", max_bytes=2)[1] == []  # live alone (2 bytes) already fails
    assert O.search_tag_values(blocks, b"a", max_bytes=0)[1] == []  # limit 0: always empty, as the reference
    # a backend block without search data: readSearchHeader fails
    nd = os.path.join(str(tmp_path), "nometa")
    os.makedirs(nd)
    assert O.block_tags(O.Block(nd))[0] == 1  # ORC_NOT_FOUND
    assert O.search_tags(blocks + [O.Block(nd)])[0] == 1
