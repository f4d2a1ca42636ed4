"""The resident search kernel (pool.hip search_resident_kernel, TSG_RESIDENT, on by default):
narrow searches served by a kernel that stays on the device and reads each query from a
mailbox slot, its records in scan order straight from the device (no host sort).

Every result is checked against the oracle (BackendSearchBlock.Search restated) through the
life cycle the host manages: queries back to back; a query after the launch left on its idle
timeout (relaunch); a block opened or closed between queries (the memory epoch forces a
relaunch, whose acquire fence sees the new columns); a query of another shape (another
template instance); a lookup between searches (the launch is ended first: it holds every
CU's LDS); a second engine on the same device (the first one's launch is ended, searches
then run as plain launches); a dense query whose records overflow the waves' LDS regions
(the segment / look-back path); and the same results with TSG_RESIDENT=0.
"""
import os
import time

import numpy as np
import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
QA = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"}, min_ms=10, max_ms=1000,
          start=T0 + 900, end=T0 + 2700)
QB = dict(tags={"http.method": "get"}, min_ms=5)
QDENSE = dict(tags={"status.code": "0"})


def request(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                           max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))


@pytest.fixture(autouse=True)
def _alone():
    """Engines other tests left for the garbage collector are finalised first: a resident
    launch runs only while its context is the only one on the device."""
    import gc
    gc.collect()


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    d = tmp_path_factory.mktemp("res")
    out = []
    for i in range(6):
        p = str(d / ("b%d" % i))
        T.synth_search_block(p, 150_000 + 40_000 * i, seed=500 + i, profile=0, encoding=T.ENC_SNAPPY,
                             page_size=256 << 10)
        out.append(p)
    return out


def expected(paths, q, limit=0):
    exp, met, st = O.search([O.Block(p) for p in paths], limit=limit, nthreads=1 if limit else 8, **q)
    assert st == 0
    return [match_key(m) for m in exp], (met["traces_inspected"], met["bytes_inspected"], met["blocks_inspected"],
                                         met["blocks_skipped"])


def got(res):
    g, met = res
    return [tsg_key(m) for m in g], (met.inspected_traces, met.inspected_bytes, met.inspected_blocks,
                                     met.skipped_blocks)


def test_back_to_back_shapes_limits_and_timing(engine, paths):
    blocks = [engine.open_block(p) for p in paths]
    c0 = engine.resident_counters()
    try:
        pa, pb = T.Pipeline(request(QA)), T.Pipeline(request(QB))
        ea, eb = expected(paths, QA), expected(paths, QB)
        ea20 = expected(paths, QA, 20)
        for rnd in range(5):
            assert got(engine.search(blocks, pa)) == ea, rnd
            assert got(engine.search(blocks, pa, flags=T.SEARCH_TIME_DEFER)) == ea, rnd  # (the span stamps)
            assert got(engine.search(blocks, pb)) == eb, rnd  # another shape: another launch
            assert got(engine.search(blocks, pa, limit=20)) == ea20, rnd
            assert got(engine.search(blocks[2:3], pa)) == expected(paths[2:3], QA)
        ks = engine.kernel_times()
        assert len(ks) == 5 and all(0 < k < 10_000_000 for k in ks), ks
        c1 = engine.resident_counters()
        assert c1["queries"] - c0["queries"] >= 20  # (served by the resident kernel)
    finally:
        for b in blocks:
            b.close()


def test_idle_exit_and_relaunch(engine, paths, monkeypatch):
    monkeypatch.setenv("TSG_RESIDENT_IDLE_US", "500")  # (read at each launch)
    blocks = [engine.open_block(p) for p in paths[:3]]  # (new blocks: the next query launches anew)
    try:
        pa = T.Pipeline(request(QA))
        e = expected(paths[:3], QA)
        c0 = engine.resident_counters()
        for gap in (0.0, 0.002, 0.0, 0.02, 0.0005, 0.0, 0.003):
            time.sleep(gap)  # (past 500 us the launch has left: the next query relaunches it)
            assert got(engine.search(blocks, pa)) == e, gap
        c1 = engine.resident_counters()
        assert c1["launches"] - c0["launches"] >= 3 and c1["queries"] - c0["queries"] == 7, (c0, c1)
    finally:
        for b in blocks:
            b.close()


def test_blocks_opened_and_closed_between_queries(engine, paths):
    pa = T.Pipeline(request(QA))
    keep = engine.open_block(paths[0])
    try:
        for i in range(1, 6):
            b = engine.open_block(paths[i])  # (new columns: the next query relaunches)
            assert got(engine.search([keep, b], pa)) == expected([paths[0], paths[i]], QA), i
            b.close()
            assert got(engine.search([keep], pa)) == expected([paths[0]], QA), i
    finally:
        keep.close()


def test_lookup_between_searches(engine, paths, tmp_path):
    ids = T.synth_v2_block(str(tmp_path / "v2"), 2000, seed=3)
    v2 = engine.open_v2block(str(tmp_path / "v2"))
    blocks = [engine.open_block(p) for p in paths[:2]]
    try:
        pa = T.Pipeline(request(QA))
        e = expected(paths[:2], QA)
        for _ in range(3):
            assert got(engine.search(blocks, pa)) == e
            hits, _ = engine.lookup([v2], np.ascontiguousarray(ids[:500]))
            assert len(hits) == 500
        assert got(engine.search(blocks, pa)) == e
    finally:
        v2.close()
        for b in blocks:
            b.close()


def test_second_engine_on_the_device(engine, paths):
    blocks = [engine.open_block(p) for p in paths[:2]]
    pa = T.Pipeline(request(QA))
    e = expected(paths[:2], QA)
    try:
        assert got(engine.search(blocks, pa)) == e  # (a resident launch of this engine)
        q0 = engine.resident_counters()["queries"]
        other = T.Engine(devices=[0])  # ends it; both now launch plain kernels
        try:
            ob = [other.open_block(p) for p in paths[:2]]
            assert got(other.search(ob, pa)) == e
            assert got(engine.search(blocks, pa)) == e
            assert engine.resident_counters()["queries"] == q0 and other.resident_counters()["queries"] == 0
            for b in ob:
                b.close()
        finally:
            other.close()
        assert got(engine.search(blocks, pa)) == e  # alone again: resident
        assert engine.resident_counters()["queries"] == q0 + 1
    finally:
        for b in blocks:
            b.close()


def test_dense_query_overflows_to_the_other_paths(engine, paths):
    blocks = [engine.open_block(p) for p in paths[:2]]
    try:
        pd = T.Pipeline(request(QDENSE))
        e = expected(paths[:2], QDENSE)
        assert len(e[0]) > 100_000
        assert got(engine.search(blocks, pd)) == e
        assert got(engine.search(blocks, T.Pipeline(request(QA)))) == expected(paths[:2], QA)
    finally:
        for b in blocks:
            b.close()


def test_resident_off_gives_the_same(paths, monkeypatch):
    monkeypatch.setenv("TSG_RESIDENT", "0")
    eng = T.Engine(devices=[0])
    try:
        blocks = [eng.open_block(p) for p in paths]
        for q in (QA, QB):
            assert got(eng.search(blocks, T.Pipeline(request(q)))) == expected(paths, q)
        for b in blocks:
            b.close()
    finally:
        eng.close()
