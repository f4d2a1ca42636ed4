"""The pipelined full scan (capi.cpp tsg_search, TSG_PIPE_DICT_MB / TSG_PIPE_BLOCKS): a full
scan with a large dictionary pass runs as consecutive launches over a few blocks each while
the host assembles the result arrays of the launches already done. The records (order and
every field) and the metrics must be those of one launch and of the oracle
(BackendSearchBlock.Search over the blocks in caller order): dense and sparse needles, a block
the header filter skips between two searched ones, a block with no match, a limit query (not
pipelined), and the same query with the pipeline off.
"""
import os

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pipe"))
    out = {}
    for name, n, seed, profile in (("hc0", 120_000, 11, 1), ("hc1", 90_000, 12, 1), ("plain", 50_000, 13, 0),
                                   ("hc2", 150_000, 14, 1)):
        p = os.path.join(d, name)
        T.synth_search_block(p, n, seed=seed, profile=profile)
        out[name] = p
    return out


def run(engine, paths, q, limit=0):
    req = T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                          max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))
    blocks = [engine.open_block(p) for p in paths]
    try:
        got, met = engine.search(blocks, T.Pipeline(req), limit=limit)
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


QUERIES = [
    dict(tags={"db.statement": "from orders", "http.url": "/carts/"}, min_ms=1),  # dense
    dict(tags={"db.statement": "where id = 77"}, start=T0 + 900, end=T0 + 2700),  # medium
    dict(tags={"db.statement": "select"}),                                          # every entry
    dict(tags={"http.url": "/api/v1/users/12"}),                                    # sparse
    dict(tags={"db.statement": "qqzz"}),                                            # absent: every block skipped
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
@pytest.mark.parametrize("per_launch", ["1", "2"])
def test_pipelined_equals_oracle_and_one_launch(engine, paths, monkeypatch, qi, per_launch):
    q = QUERIES[qi]
    order = [paths["hc0"], paths["plain"], paths["hc1"], paths["hc2"]]  # (plain: skipped by the header filter)
    exp = oracle(order, q)
    monkeypatch.setenv("TSG_PIPE_DICT_MB", "0")
    assert run(engine, order, q) == exp  # one launch
    monkeypatch.setenv("TSG_PIPE_DICT_MB", "1")
    monkeypatch.setenv("TSG_PIPE_SPARSE", "1")
    monkeypatch.setenv("TSG_PIPE_BLOCKS", per_launch)
    assert run(engine, order, q) == exp  # pipelined
    # a limit query is never pipelined; its result is the oracle's consumer
    assert run(engine, order, q, limit=20) == oracle(order, q, limit=20)


def test_pipelined_repeat_and_one_block(engine, paths, monkeypatch):
    monkeypatch.setenv("TSG_PIPE_DICT_MB", "1")
    monkeypatch.setenv("TSG_PIPE_SPARSE", "1")
    monkeypatch.setenv("TSG_PIPE_BLOCKS", "1")
    q = QUERIES[0]
    order = [paths["hc2"], paths["hc0"], paths["hc1"]]
    exp = oracle(order, q)
    for _ in range(3):  # (reused result holders and device outputs)
        assert run(engine, order, q) == exp
    assert run(engine, [paths["hc1"]], q) == oracle([paths["hc1"]], q)  # one block: one launch
