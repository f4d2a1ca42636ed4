"""WAL search blocks (StreamingSearchBlock) on the CPU: the oracle's restatement of
replay + dedupe/combine + search pinned to the reference's own known answers
(tempodb/search/streaming_search_block_test.go), and the engine's flatbuffer writer
cross-checked against the oracle's independent restatement of the Go builder.
CPU only (the engine side of these blocks is tests/test_gpu_wal.py)."""
import os
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import gen_search_data, ref_id

REF_TAGS = {"key1": ["value10", "value11"], "key2": ["value20", "value21"],
            "key3": ["value30", "value31"], "key4": ["value40", "value41"]}


def wal(tmp_path, entries, enc=T.ENC_SNAPPY, name=None):
    p = os.path.join(str(tmp_path), name or T.wal_filename(enc))
    T.write_wal_search(p, entries, enc)
    return p


# newStreamingSearchBlockWithTraces + TestStreamingSearchBlockReplay (:26-95), both encodings we read
@pytest.mark.parametrize("enc", [T.ENC_NONE, T.ENC_SNAPPY])
def test_replay_matches_every_trace(tmp_path, enc):
    p = wal(tmp_path, [{"id": ref_id(i, 8), "tags": REF_TAGS} for i in range(100)], enc)
    m, met, st = O.search([O.Block(p, wal=True)], tags={"key1": "value10"})
    assert st == 0 and len(m) == 100


# TestStreamingSearchBlockSearchBlock (:97-155)
@pytest.mark.parametrize("tags,results,inspected,traces,skipped", [
    ({"key1": "value10"}, 10, 1, 10, 0),
    ({"nomatch": "nomatch"}, 0, 0, 0, 1),
])
def test_search_block_known_answers(tmp_path, tags, results, inspected, traces, skipped):
    p = wal(tmp_path, [{"id": ref_id(i, 8), "tags": REF_TAGS} for i in range(10)], T.ENC_NONE)
    m, met, st = O.search([O.Block(p, wal=True)], tags=tags)
    assert (len(m), met["blocks_inspected"], met["traces_inspected"], met["blocks_skipped"]) == \
        (results, inspected, traces, skipped)


# TestStreamingSearchBlockIteratorDedupes (:157-205): 1000 appends of one id combine to one entry
def test_iterator_dedupes(tmp_path):
    tid = bytes(range(16))
    p = wal(tmp_path, [{"id": tid, "tags": gen_search_data(i)} for i in range(1000)], T.ENC_NONE)
    m, met, st = O.search([O.Block(p, wal=True)], tags={"key10": "value_A_10", "key20": "value_B_20"})
    assert st == 0 and len(m) == 1 and met["traces_inspected"] == 1
    # bytesInspected = the combined entry's length (SearchEntryMutable.ToBytes of the union)
    union = {"id": tid, "tags": {}}
    for i in range(1000):
        union["tags"].update(gen_search_data(i))
    assert met["bytes_inspected"] == len(O.entry_to_bytes(union)) == len(T.fb_search_entry(union))


def test_block_filter_is_exact_value_contains(tmp_path):
    """The mutable header's Contains is a map lookup (searchdatamap.go:43-49): a substring
    that would match every entry skips the whole WAL block."""
    p = wal(tmp_path, [{"id": ref_id(i), "tags": REF_TAGS} for i in range(5)])
    m, met, _ = O.search([O.Block(p, wal=True)], tags={"key1": "value1"})
    assert len(m) == 0 and met["blocks_skipped"] == 1
    m, met, _ = O.search([O.Block(p, wal=True)], tags={"key1": "value11"})
    assert len(m) == 5


def test_mixed_case_keys_follow_binary_search(tmp_path):
    """Keys sorted by original case then lowercased (searchdatamap.go:74-109) can leave an
    entry's vector out of order; FindTag's binary search then misses a key (pitfall P3)."""
    # {"B", "a"}: sorted "B" < "a", prepended -> vector ["a", "b"] (ascending: violates descending)
    e = {"id": ref_id(1), "tags": {"B": ["x"], "a": ["y"]}}
    fb = T.fb_search_entry(e)
    assert O.contains_tag_entry(fb, b"b", b"x") and not O.contains_tag_entry(fb, b"a", b"y")
    p = wal(tmp_path, [e])
    assert len(O.search([O.Block(p, wal=True)], tags={"b": "x"})[0]) == 1
    m, met, _ = O.search([O.Block(p, wal=True)], tags={"a": "y"})  # header has it, the entry search misses it
    assert len(m) == 0 and met["blocks_inspected"] == 1 and met["traces_inspected"] == 1


def test_partial_replay_keeps_pages_before_damage(tmp_path):
    ents = [{"id": ref_id(i), "tags": REF_TAGS} for i in range(6)]
    p = wal(tmp_path, ents, T.ENC_NONE)
    full = open(p, "rb").read()
    with open(p, "wb") as f:
        f.write(full[:len(full) - 7])  # tear the last page
    m, met, _ = O.search([O.Block(p, wal=True)], tags={"key1": "value10"})
    assert len(m) == 5 and met["traces_inspected"] == 5


def test_wal_filename_rules(tmp_path):
    good = wal(tmp_path, [{"id": ref_id(0), "tags": REF_TAGS}])
    O.Block(good, wal=True)
    for bad in ["nouuid:t:v2:snappy", "1c505e8b-26cd-4621-ba7d-792bb55282d5::v2:snappy",
                "1c505e8b-26cd-4621-ba7d-792bb55282d5:t:v2:bogus", "1c505e8b-26cd-4621-ba7d-792bb55282d5:t:v2"]:
        with pytest.raises(OSError):
            O.Block(os.path.join(str(tmp_path), bad), wal=True)


@pytest.mark.parametrize("seed", range(4))
def test_writer_matches_oracle_builder(seed):
    """The engine's SearchEntryMutable.ToBytes restatement (writer.cpp) and the oracle's
    (tsg_oracle.c, written separately from vendor/.../flatbuffers/go/builder.go) agree
    byte for byte: mixed case, shared strings, duplicate values after lowercasing."""
    rng = random.Random(seed)
    alpha = ["a", "B", "c", "Key", "key", "VAL", "val", "Été", "x.y", ""]
    for _ in range(200):
        tags = {}
        for _k in range(rng.randrange(0, 7)):
            k = "".join(rng.choice(alpha) for _ in range(rng.randrange(1, 3)))
            tags[k] = sorted({"".join(rng.choice(alpha) for _ in range(rng.randrange(0, 3)))
                              for _ in range(1 + rng.randrange(3))})
        e = {"id": bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 8, 16]))),
             "start": rng.choice([0, rng.getrandbits(63)]), "end": rng.choice([0, rng.getrandbits(63)]), "tags": tags}
        assert T.fb_search_entry(e) == O.entry_to_bytes(e), e
