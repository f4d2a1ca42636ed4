"""The resident search kernel, round 6 (pool.hip search_resident_kernel and its host side):

- long runs: a workgroup whose unit run is longer than two units per thread (> 1536 units:
  the ordered-output prefix sum takes more than one pass), forced with TSG_GROUPS=8;
- the exact mailbox check: a slot written torn (two words moved by +-d, the plain sum unchanged,
  which round 5's additive checksum accepted) is re-read, not run (tsg_debug_set "res_torn");
- queries in flight at once: concurrent callers and tsg_search_batch post while earlier queries
  run (each holds its own result area); every result against the oracle, the batch's resident
  launch timed by its dispatch timestamps;
- the XCD-weighted split gives the same records as even runs, and tsg_metrics.path names the
  kernels that served a search.
"""
import faulthandler
import os
import signal
import threading
import time

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, tsg_key

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
QA = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"}, min_ms=10, max_ms=1000,
          start=T0 + 900, end=T0 + 2700)
QB = dict(tags={"http.method": "get"}, min_ms=5)
QC = dict(tags={"service.name": "svc-11"}, max_ms=200)


def request(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                           max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))


@pytest.fixture(autouse=True)
def _alone():
    import gc
    gc.collect()


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    d = tmp_path_factory.mktemp("res2")
    out = []
    for i in range(7):
        p = str(d / ("b%d" % i))
        T.synth_search_block(p, 1_000_000 if i < 6 else 300_000, seed=700 + i, profile=0, encoding=T.ENC_SNAPPY)
        out.append(p)
    return out


_exp_cache = {}


def expected(paths, q, limit=0):
    key = (tuple(paths), repr(sorted(q.items())), limit)
    if key not in _exp_cache:
        exp, met, st = O.search([O.Block(p) for p in paths], limit=limit, nthreads=1 if limit else 8, **q)
        assert st == 0
        _exp_cache[key] = ([match_key(m) for m in exp], (met["traces_inspected"], met["bytes_inspected"],
                                                          met["blocks_inspected"], met["blocks_skipped"]))
    return _exp_cache[key]


def got(res):
    g, met = res
    return [tsg_key(m) for m in g], (met.inspected_traces, met.inspected_bytes, met.inspected_blocks,
                                     met.skipped_blocks)


def test_runs_longer_than_two_units_per_thread(engine, paths):
    """8 workgroups over 6.3 M entries: ~1540 units each, past the 1536 a single prefix pass
    covered (the records of units beyond it would have been read from the wrong LDS slots)."""
    blocks = [engine.open_block(p) for p in paths]
    T.debug_set("groups", 8)
    try:
        n = sum(b.info()["entries"] for b in blocks)
        assert n // 512 // 8 > 1536, n
        qa2 = dict(QA, tags={"service.name": "svc-21", "http.method": "post", "status.code": "error"})
        for q in (QA, qa2):
            res = engine.search(blocks, T.Pipeline(request(q)))
            assert got(res) == expected(paths, q)
            assert res[1].path & T.PATH_RESIDENT, res[1].path
    finally:
        T.debug_set("groups", 0)
        for b in blocks:
            b.close()


def test_torn_slot_is_reread(engine, paths):
    blocks = [engine.open_block(p) for p in paths[:3]]
    try:
        pa = T.Pipeline(request(QA))
        e = expected(paths[:3], QA)
        assert got(engine.search(blocks, pa)) == e  # (the resident launch is up)
        c0 = engine.resident_counters()
        for _ in range(3):
            T.debug_set("res_torn", 1)
            res = engine.search(blocks, pa)
            assert got(res) == e  # (the torn range words would have matched nothing)
            assert res[1].path & T.PATH_RESIDENT
        c1 = engine.resident_counters()
        assert c1["rejects"] > c0["rejects"], (c0, c1)
        assert c1["queries"] - c0["queries"] == 3 and c1["launches"] == c0["launches"], (c0, c1)
    finally:
        T.debug_set("res_torn", 0)
        for b in blocks:
            b.close()


def test_concurrent_callers_share_the_resident_launch(engine, paths):
    """Threads with different queries and block sets search at once: each posts while the
    others' queries run; every result is the oracle's."""
    blocks = [engine.open_block(p) for p in paths]
    sets = [blocks[:3], blocks[3:6], blocks[1:5], blocks[6:]]
    psets = [paths[:3], paths[3:6], paths[1:5], paths[6:]]
    # (QB narrowed: its dense form's hundreds of thousands of records per search were unpacked
    # into Python objects under the GIL, 6 threads x 12 searches, past the join's bound)
    qs = [QA, dict(QB, tags={"http.method": "get", "status.code": "error"}), QC]
    pipes = [T.Pipeline(request(q)) for q in qs]
    exp = {(s, k): expected(psets[s], qs[k]) for s in range(len(sets)) for k in range(len(qs))}
    errors = []
    c0 = engine.resident_counters()

    def worker(t):
        try:
            for r in range(12):
                s, k = (t + r) % len(sets), (t * 7 + r) % len(qs)
                assert got(engine.search(sets[s], pipes[k])) == exp[(s, k)], (t, r, s, k)
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    th = [threading.Thread(target=worker, args=(t,), daemon=True) for t in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join(150)
    hung = [x for x in th if x.is_alive()]
    if hung:
        # (the blocks stay open: a caller still inside tsg_search uses them). With
        # TSG_SEGV_TRACE=1 each hung caller prints its native stack (libtsg's SIGUSR2 handler)
        if os.environ.get("TSG_SEGV_TRACE"):
            for x in hung:
                signal.pthread_kill(x.ident, signal.SIGUSR2)
            time.sleep(1)
            faulthandler.dump_traceback(all_threads=True)
        pytest.fail("%d callers never returned; resident counters %s -> %s" % (len(hung), c0, engine.resident_counters()))
    try:
        assert not errors, errors[0]
        c1 = engine.resident_counters()
        assert c1["queries"] - c0["queries"] >= 72, (c0, c1)
    finally:
        for b in blocks:
            b.close()


def test_search_batch(engine, paths):
    blocks = [engine.open_block(p) for p in paths[:6]]
    clones = [[b.clone(engine) for b in blocks] for _ in range(2)]
    try:
        pa, pc = T.Pipeline(request(QA)), T.Pipeline(request(QC))
        ea, ec = expected(paths[:6], QA), expected(paths[:6], QC)
        sets = [blocks] + clones
        items = [(sets[i % 3], pa) for i in range(64)]
        res, dns = engine.search_batch(items, depth=8)
        assert len(res) == 64
        for r in res:
            assert got(r) == ea
            assert r[1].path == T.PATH_RESIDENT
        # one resident launch served the batch: its dispatch time is the batch's device time
        assert 0 < dns < 64 * 2_000_000, dns
        mixed = [(sets[i % 3], pa if i % 2 else pc) + ((20,) if i % 5 == 0 else ()) for i in range(40)]
        res, _ = engine.search_batch(mixed, depth=6)
        for i, r in enumerate(res):
            q = QA if i % 2 else QC
            assert got(r) == expected(paths[:6], q, 20 if i % 5 == 0 else 0), i
        # counts only (what the bench's batched leg reads)
        res, dns = engine.search_batch(items[:16], depth=4, unpack=False)
        assert all(n == len(ea[0]) for n, _ in res) and dns > 0
    finally:
        for s in clones:
            for b in s:
                b.close()
        for b in blocks:
            b.close()


def test_xsplit_matches_even_runs(engine, paths):
    """The XCD-weighted split (after its calibration samples) and even runs give the same
    records and metrics."""
    blocks = [engine.open_block(p) for p in paths[:6]]
    T.debug_set("xsplit", 1)
    try:
        pa = T.Pipeline(request(QA))
        e = expected(paths[:6], QA)
        s0 = engine.resident_counters()["xsplit_samples"]
        for _ in range(24):
            assert got(engine.search(blocks, pa)) == e
        assert engine.resident_counters()["xsplit_samples"] > s0
        T.debug_set("xsplit", 0)
        s1 = engine.resident_counters()["xsplit_samples"]
        for _ in range(3):
            assert got(engine.search(blocks, pa)) == e
        assert engine.resident_counters()["xsplit_samples"] == s1
    finally:
        T.debug_set("xsplit", 0)
        for b in blocks:
            b.close()


def test_metrics_path(engine, paths, monkeypatch):
    blocks = [engine.open_block(p) for p in paths[:2]]
    try:
        _, m = engine.search(blocks, T.Pipeline(request(QA)))
        assert m.path == T.PATH_RESIDENT
        _, m = engine.search(blocks, T.Pipeline(request(dict(tags={"status.code": "0"}))))
        assert m.path & T.PATH_OTHER  # (dense: the records overflow to the look-back path)
    finally:
        for b in blocks:
            b.close()
    monkeypatch.setenv("TSG_RESIDENT", "0")
    eng = T.Engine(devices=[0])
    try:
        blocks = [eng.open_block(p) for p in paths[:2]]
        _, m = eng.search(blocks, T.Pipeline(request(QA)))
        assert m.path == T.PATH_PLAIN
        for b in blocks:
            b.close()
    finally:
        eng.close()
