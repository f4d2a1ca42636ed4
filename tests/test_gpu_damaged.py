"""GPU parity on damaged blocks: BackendSearchBlock.Search's error paths
(tempodb/search/backend_search_block.go:247-266).

* A failing index record ends the block SILENTLY: `record, _ := ir.At(ctx, i)` drops the
  error and `record == nil` returns nil (:252-255). Pages before it are searched.
* A damaged data page k returns an error from Search AFTER the matches of pages < k have
  been sent (:258-266); the ingester logs it and keeps everything else
  (modules/ingester/instance_search.go:179-182).

The engine decodes at open, so it keeps the pages the reference would reach and reports
the data-page error per block (tsg_result.block_status). Matches, metrics and per-block
status must equal the oracle's sequential restatement.
"""
import random

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import (damage_data_page, damage_index_page_checksum, gen_search_data, match_key,
                           random_entries, ref_id, repage_index, tsg_key, write_block, zero_index_record)

pytestmark = pytest.mark.gpu


def run(engine, paths, limit=0, **q):
    req = T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                          max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))
    blocks = [engine.open_block(p) for p in paths]
    try:
        infos = [b.info() for b in blocks]
        got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
    finally:
        for b in blocks:
            b.close()
    exp, omet, _ = O.search([O.Block(p) for p in paths], limit=limit, **q)
    assert [tsg_key(m) for m in got] == [match_key(m) for m in exp]
    assert (met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks) == (
        omet["traces_inspected"], omet["bytes_inspected"], omet["blocks_inspected"], omet["blocks_skipped"])
    assert met.block_status == omet["block_status"]
    return got, met, infos


def three_blocks(tmp_path, enc, n=1500, page_size=4096):
    rng = random.Random(enc * 7 + n)
    paths = []
    for b in range(3):
        ents = random_entries(rng, n, nkeys=3, nvals=4)
        paths.append(write_block(str(tmp_path), "b%d" % b, ents, enc, page_size=page_size))
    return paths


QUERIES = [dict(tags={"k0": "v"}), dict(tags={"k1": "v1"}, min_ms=5), dict()]


@pytest.mark.parametrize("enc,how", [(T.ENC_SNAPPY, "payload"), (T.ENC_SNAPPY, "truncate"),
                                     (T.ENC_NONE, "length"), (T.ENC_NONE, "objlen")])
def test_damaged_data_page_keeps_earlier_matches(engine, tmp_path, enc, how):
    paths = three_blocks(tmp_path, enc)
    k = 7
    damage_data_page(paths[1], k, how)
    for q in QUERIES:
        got, met, infos = run(engine, paths, **q)
        assert met.block_status == [0, T.TSG_E_CORRUPT, 0]
        assert met.block_errors[1]
        assert infos[1]["stop_status"] == T.TSG_E_CORRUPT and infos[1]["pages"] == k
        assert any(m.block_idx == 2 for m in got) or not q  # the block after it is still searched
    # a limit reached before the damaged page: Search quits first, no error
    got, met, _ = run(engine, paths, limit=3, tags={"k0": "v"})
    assert met.block_status == [0, 0, 0]
    # a limit the blocks cannot satisfy: the damaged block reports its error
    got, met, _ = run(engine, paths, limit=100000, tags={"k0": "v"})
    assert met.block_status == [0, T.TSG_E_CORRUPT, 0]


def test_damaged_first_page(engine, tmp_path):
    paths = three_blocks(tmp_path, T.ENC_SNAPPY)
    damage_data_page(paths[0], 0, "payload")
    for q in QUERIES:
        got, met, infos = run(engine, paths, **q)
        assert infos[0]["entries"] == 0 and met.block_status == [T.TSG_E_CORRUPT, 0, 0]


@pytest.mark.parametrize("enc", [T.ENC_NONE, T.ENC_SNAPPY])
def test_damaged_index_ends_block_silently(engine, tmp_path, enc):
    paths = three_blocks(tmp_path, enc)
    repage_index(paths[0], 4)  # 4 records per index page: page k > 0 exists
    repage_index(paths[1], 4)
    damage_index_page_checksum(paths[0], 2)  # records 8.. unreachable
    zero_index_record(paths[1], 5)           # At(5) fails: pages 0..4 searched
    for q in QUERIES:
        got, met, infos = run(engine, paths, **q)
        assert met.block_status == [0, 0, 0]
        assert infos[0]["pages"] == 8 and infos[0]["index_truncated"] == 1
        assert infos[1]["pages"] == 5 and infos[1]["index_truncated"] == 1
    for lim in (1, 50, 5000):
        run(engine, paths, limit=lim, tags={"k0": "v"})


def test_damaged_index_first_page(engine, tmp_path):
    """Index page 0 fails its checksum: no record is reachable, the block inspects only
    its header bytes (was rejected at open before round 2)."""
    ents = [{"id": ref_id(i), "tags": gen_search_data(i)} for i in range(2000)]
    p = write_block(str(tmp_path), "c", ents, page_size=4096)
    damage_index_page_checksum(p, 0)
    got, met, infos = run(engine, [p], tags={"key20": "value"})
    assert got == [] and met.inspected_traces == 0 and met.inspected_blocks == 1
    assert infos[0]["entries"] == 0 and infos[0]["index_truncated"] == 1
