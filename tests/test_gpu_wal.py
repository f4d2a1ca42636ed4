"""GPU parity for WAL search blocks (StreamingSearchBlock): libtsg's replay into a
resident block + the HIP search vs the oracle's restatement, bit-exact (ordered
matches, metrics), incl. duplicates combined at replay, mixed-case keys that break
the descending key order (FindTag's binary search decides), exact-value block
filter, limits, a torn last page, and WAL + backend blocks in one search."""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import gen_search_data, match_key, random_entries, ref_id, tsg_key, write_block
from tests.test_gpu_search import assert_parity

pytestmark = pytest.mark.gpu

REF_TAGS = {"key1": ["value10", "value11"], "key2": ["value20", "value21"],
            "key3": ["value30", "value31"], "key4": ["value40", "value41"]}


def wal(tmp_path, entries, enc=T.ENC_SNAPPY, name=None):
    p = os.path.join(str(tmp_path), name or T.wal_filename(enc))
    T.write_wal_search(p, entries, enc)
    return p


def both(engine, paths, wal_flags, tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=0):
    req = T.SearchRequest(tags=dict(tags or {}), min_duration_ms=min_ms, max_duration_ms=max_ms, start=start,
                          end=end)
    blocks = [engine.open_wal_block(p) if w else engine.open_block(p) for p, w in zip(paths, wal_flags)]
    got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
    oblocks = [O.Block(p, wal=w) for p, w in zip(paths, wal_flags)]
    exp, omet, st = O.search(oblocks, tags=tags, min_ms=min_ms, max_ms=max_ms, start=start, end=end, limit=limit)
    assert st == 0
    for b in blocks:
        b.close()
    return got, met, exp, omet


@pytest.mark.parametrize("enc", [T.ENC_NONE, T.ENC_SNAPPY])
def test_reference_known_answers(engine, tmp_path, enc):
    p = wal(tmp_path, [{"id": ref_id(i, 8), "tags": REF_TAGS} for i in range(10)], enc)
    got, met, exp, omet = both(engine, [p], [True], tags={"key1": "value10"})
    assert len(got) == 10 and met.inspected_blocks == 1 and met.inspected_traces == 10
    assert_parity(got, met, exp, omet)
    got, met, exp, omet = both(engine, [p], [True], tags={"nomatch": "nomatch"})
    assert len(got) == 0 and met.skipped_blocks == 1
    assert_parity(got, met, exp, omet)


def test_dedupe_combines(engine, tmp_path):
    tid = bytes(range(16))
    p = wal(tmp_path, [{"id": tid, "tags": gen_search_data(i)} for i in range(1000)], T.ENC_NONE)
    got, met, exp, omet = both(engine, [p], [True], tags={"key10": "value_A_10", "key20": "value_B_20"})
    assert len(got) == 1 and met.inspected_traces == 1
    assert_parity(got, met, exp, omet)
    info = engine.open_wal_block(p).info()
    assert info["streaming"] == 1 and info["entries"] == 1 and info["partial"] == 0


def random_wal_entries(rng, n, dup_frac=0.3, mixed_case=True):
    ents = random_entries(rng, n, nkeys=6, nvals=6, multi=3)
    out = []
    for e in ents:
        if mixed_case and rng.random() < 0.2:  # original-case keys: order broken after lowercasing
            e["tags"]["K%d" % rng.randrange(6)] = ["v%d-x" % rng.randrange(6)]
            e["tags"]["Zz"] = ["top"]
        out.append(e)
        while rng.random() < dup_frac:  # the same trace appended again with more data
            d = {"id": e["id"], "start": e["start"] - rng.randrange(10**9) if e["start"] else 0,
                 "end": e["end"] + rng.randrange(10**9) if e["end"] else 0,
                 "tags": {"k%d" % rng.randrange(6): ["v%d-y" % rng.randrange(6)]}}
            out.append(d)
    rng.shuffle(out)  # append order != id order: replay sorts
    return out


@pytest.mark.parametrize("seed", range(3))
def test_random_parity(engine, tmp_path, seed):
    rng = random.Random(seed)
    p = wal(tmp_path, random_wal_entries(rng, 3000), T.ENC_SNAPPY if seed % 2 else T.ENC_NONE)
    t0 = 1_700_000_000
    queries = [
        dict(tags={"k1": "v2-x"}),
        dict(tags={"k1": "v2-x", "k3": "v1-z"}),
        dict(tags={"k0": "v3-y"}, min_ms=5, max_ms=5000),
        dict(tags={"zz": "top"}),
        dict(tags={"k2": "v4-x"}, start=t0 + 600, end=t0 + 2400),
        dict(min_ms=100),
        dict(tags={"root.service.name": "svc-1"}),
        dict(tags={"k1": "v"}),  # substring: the exact-value block filter skips the block
    ]
    for q in queries:
        for limit in (0, 7):
            got, met, exp, omet = both(engine, [p], [True], limit=limit, **q)
            assert_parity(got, met, exp, omet)


def test_torn_last_page(engine, tmp_path):
    p = wal(tmp_path, [{"id": ref_id(i), "tags": REF_TAGS} for i in range(6)], T.ENC_NONE)
    full = open(p, "rb").read()
    with open(p, "wb") as f:
        f.write(full[:-7])
    blk = engine.open_wal_block(p)
    assert blk.info()["partial"] == 1 and blk.info()["entries"] == 5
    blk.close()
    got, met, exp, omet = both(engine, [p], [True], tags={"key1": "value10"})
    assert len(got) == 5
    assert_parity(got, met, exp, omet)


def test_empty_wal_is_not_found(engine, tmp_path):
    p = os.path.join(str(tmp_path), T.wal_filename(T.ENC_NONE))
    open(p, "wb").close()
    with pytest.raises(T.TsgError):
        engine.open_wal_block(p)


def test_wal_and_backend_blocks_together(engine, tmp_path):
    rng = random.Random(7)
    bp = write_block(str(tmp_path), "b", random_entries(rng, 2000))
    wp = wal(tmp_path, random_wal_entries(rng, 2000, mixed_case=False))
    for limit in (0, 25):
        got, met, exp, omet = both(engine, [wp, bp, wp], [True, False, True], tags={"k2": "v3-x"}, limit=limit)
        assert_parity(got, met, exp, omet)


def test_tags_and_values(engine, tmp_path):
    p = wal(tmp_path, [{"id": ref_id(i), "tags": {"a": ["x%d" % (i % 3)], "b": ["y"]}} for i in range(9)])
    blk = engine.open_wal_block(p)
    assert sorted(blk.tags()) == [b"a", b"b"]
    assert sorted(blk.tag_values(b"a")) == [b"x0", b"x1", b"x2"]
    assert blk.tag_values(b"zz") == []
    blk.close()
