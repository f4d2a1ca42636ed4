"""dict_stream_kernel (search.hip): bytes.Contains over large dictionaries as one byte
stream — the config-4 path (long db.statement / http.url values).

ContainsTag matches a term when the needle is a substring of one of the entry's values
for the key (pkg/tempofb/searchdata_util.go:47-61, bytes.Contains). The stream kernel
scans a key's value bytes back to back, so these tests aim at what that could get wrong:
needles of 1, 2, 3, 4 and many bytes (the SWAR prefilter takes two), needles up to the
1024-byte window limit and one past it (the lane-per-value path), matches that would
straddle two values (must not count), values shorter than the needle, empty values,
matches at a value's first and last byte, window (1 KiB) and wave span (64 KiB)
boundaries, single-valued keys (identity: value = set) and multi-valued ones (a set
matches when any value does). Expected: the oracle; and the lane-per-value engine
(TSG_DICT_STREAM=0) must agree record for record.
"""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key, write_block

pytestmark = pytest.mark.gpu

ALPHA = "abcd e"


def _value(rng, n):
    return "".join(rng.choice(ALPHA) for _ in range(n))


@pytest.fixture(scope="module")
def dict_blocks(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dstream"))
    rng = random.Random(1234)
    paths, long_vals = [], []
    for b in range(2):
        ents = []
        ids = sorted({bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(2500)})
        for i, tid in enumerate(ids):
            r = rng.random()
            n = 0 if r < 0.02 else rng.randrange(1, 12) if r < 0.12 else rng.randrange(100, 3000)
            st = _value(rng, n)
            if n > 1100:
                long_vals.append(st)
            tags = {"db.statement": [st], "root.service.name": ["svc-%d" % (i % 3)]}
            if rng.random() < 0.7:
                tags["multi"] = sorted({_value(rng, rng.randrange(20, 900)) for _ in range(1 + rng.randrange(3))})
            start = 1_700_000_000 * 10**9 + rng.randrange(3600 * 10**9)
            ents.append({"id": tid, "start": start, "end": start + rng.randrange(1, 10**9), "tags": tags})
        paths.append(write_block(d, "b%d" % b, ents, page_size=256 << 10))
    return paths, long_vals


def needles(long_vals):
    rng = random.Random(99)
    out = ["a", "e", " ", "ab", "d ", "abc", "abca", "cab e", "no-such-needle", "abcdeabcde" * 3]
    for _ in range(24):
        v = rng.choice(long_vals)
        n = rng.choice([2, 3, 5, 8, 17, 40, 100])
        k = rng.randrange(len(v) - n)
        out.append(v[k:k + n])
    v = long_vals[0]
    out += [v[:5], v[-5:], v[:1000], v[50:1074], v[:1024], v[10:1035]]  # first/last bytes, 1000, 1024, 1025
    return out


def check(eng, blocks, paths, tags):
    got, met = eng.search(blocks, T.Pipeline(T.SearchRequest(tags=tags)))
    exp, omet, st = O.search([O.Block(p) for p in paths], tags=tags, nthreads=2)
    assert st == 0
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp], tags
    assert (met.inspected_traces, met.inspected_bytes) == (omet["traces_inspected"], omet["bytes_inspected"])
    return [tsg_key(m) for m in got]


def test_stream_matches_oracle(engine, dict_blocks):
    paths, long_vals = dict_blocks
    blocks = [engine.open_block(p) for p in paths]
    try:
        total = 0
        for nd in needles(long_vals):
            for key in ("db.statement", "multi"):
                total += len(check(engine, blocks, paths, {key: nd}))
        assert total > 0
    finally:
        for b in blocks:
            b.close()


def test_stream_two_terms_and_lane_path_agree(engine, dict_blocks):
    paths, long_vals = dict_blocks
    os.environ["TSG_DICT_STREAM"] = "0"
    try:
        lane = T.Engine()
    finally:
        del os.environ["TSG_DICT_STREAM"]
    ba = [engine.open_block(p) for p in paths]
    bb = [lane.open_block(p) for p in paths]
    try:
        rng = random.Random(7)
        for nd in needles(long_vals)[:20]:
            tags = {"db.statement": nd, "multi": rng.choice(["ab", "c", "dd e", "eeee"])}
            assert check(engine, ba, paths, tags) == check(lane, bb, paths, tags)
    finally:
        for b in ba + bb:
            b.close()
        lane.close()


def test_stream_every_start_a_candidate(engine, tmp_path):
    """Values that are long runs of one byte: with the needle "aa" every start of a KiB is a
    candidate (1024 per step: the wave's whole candidate list, flushed before the next step
    appends), "aab" makes them all fail verification but the last, and "ba" sits at run
    boundaries."""
    rng = random.Random(5)
    ents = []
    ids = sorted({bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(1500)})
    for i, tid in enumerate(ids):
        n = rng.randrange(200, 3000)
        st = "a" * n if i % 3 else "a" * (n // 2) + "b" + "a" * (n // 2)
        start = 1_700_000_000 * 10**9 + rng.randrange(3600 * 10**9)
        ents.append({"id": tid, "start": start, "end": start + 1000, "tags": {"db.statement": [st]}})
    path = write_block(str(tmp_path), "runs", ents, page_size=256 << 10)
    blk = engine.open_block(path)
    try:
        for nd in ("aa", "aaa", "aab", "ba", "aaaaaaaaaaaaaaaaaaaab", "a" * 300):
            assert check(engine, [blk], [path], {"db.statement": nd})
    finally:
        blk.close()


@pytest.mark.parametrize("mode", [1, 0, 2])
def test_bitmap_mode_and_dead_terms(engine, dict_blocks, mode):
    """Full scans on the dictionary-pass path return one bit per entry (bitmap mode, 1 / auto 2
    after a dense query) or 8-byte positions (0): the same records and metrics as the oracle;
    limit queries keep positions. A term no dictionary value matches skips its block's scan on
    the device (needle absent in one block, in both, and a second term absent)."""
    paths, long_vals = dict_blocks
    blocks = [engine.open_block(p) for p in paths]
    T.debug_set("lb_bitmap", mode)
    try:
        for tags in ({"db.statement": "a"}, {"db.statement": "e"}, {"multi": "ab"}, {"db.statement": "cab e"},
                     {"db.statement": long_vals[0][:40]}, {"db.statement": "no-such-needle"},
                     {"db.statement": "a", "multi": "no-such-needle"}, {"db.statement": "d ", "multi": "c"}):
            check(engine, blocks, paths, tags)
        got, met = engine.search(blocks, T.Pipeline(T.SearchRequest(tags={"db.statement": "a"})), limit=7)
        exp, omet, st = O.search([O.Block(p) for p in paths], tags={"db.statement": "a"}, limit=7)
        assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
        # the needle in one block only: the other block's scan is skipped, its metrics still count
        only = long_vals[0][100:140]
        check(engine, blocks, paths, {"db.statement": only})
    finally:
        T.debug_set("lb_bitmap", 2)
        for b in blocks:
            b.close()
