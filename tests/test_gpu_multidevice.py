"""One process, several device contexts (the single-process shard manager, one HIP
stream and host thread per device; the ingester's goroutine per block,
modules/ingester/instance_search.go:164-185): tsg_search groups the blocks per device, fans the
parts out (capi.cpp fan_out) and merges the per-device records in caller block order — limit 0,
limit waves across devices, a header-skipped block between searched ones, a dense query whose
records overflow to the look-back path on every device. Two contexts on ordinal 0 stand in for
two GPUs on the one-GPU box (their resident launches are off: two contexts share the device).

And another process on the same GPU: while it holds a libtsg context there, this
process's narrow searches launch plainly (tsg_metrics.path has PATH_COTENANT), and once it has
gone they return to the resident kernel.
"""
import os
import subprocess
import sys
import time

import pytest

from oracle import oracle as O
import tempo_amd as T
from tests.helpers import match_key, random_entries, tsg_key, write_block

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
QA = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"}, min_ms=10, max_ms=1000,
          start=T0 + 900, end=T0 + 2700)
QB = dict(tags={"service.name": "svc-03"}, min_ms=2)
QDENSE = dict(tags={"status.code": "0"})


def request(q):
    return T.SearchRequest(tags=dict(q.get("tags", {})), min_duration_ms=q.get("min_ms", 0),
                           max_duration_ms=q.get("max_ms", 0), start=q.get("start", 0), end=q.get("end", 0))


@pytest.fixture(autouse=True)
def _alone():
    import gc
    gc.collect()


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    import random
    d = tmp_path_factory.mktemp("mdev")
    out = []
    for i in range(6):
        p = str(d / ("b%d" % i))
        T.synth_search_block(p, 120_000 + 30_000 * i, seed=900 + i, profile=0, encoding=T.ENC_SNAPPY,
                             page_size=256 << 10)
        out.append(p)
    # a block without the query's keys: MatchesBlock skips it from its header
    out.insert(3, write_block(str(d), "noservice", random_entries(random.Random(5), 3000, with_names=True)))
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


def test_search_across_device_contexts(paths):
    eng = T.Engine(devices=[0, 0])
    assert eng.device_count == 2
    blocks = [eng.open_block(p, device=i % 2) for i, p in enumerate(paths)]
    try:
        assert [b.info()["device"] for b in blocks] == [0] * len(blocks)  # (both contexts: ordinal 0)
        for q in (QA, QB):
            pl = T.Pipeline(request(q))
            for limit in (0, 20, 300):
                e = expected(paths, q, limit)
                res = eng.search(blocks, pl, limit=limit)
                assert got(res) == e, (q, limit)
                if not limit:
                    assert e[1][3] == 1  # (the keyless block was skipped by its header)
        # the same blocks in another order: the merge follows the caller's block order
        rev = blocks[::-1]
        assert got(eng.search(rev, T.Pipeline(request(QA)))) == expected(paths[::-1], QA)
        # dense: every device's records overflow the pool kernels' LDS buffers (look-back path)
        e = expected(paths, QDENSE)
        assert len(e[0]) > 500_000
        res = eng.search(blocks, T.Pipeline(request(QDENSE)))
        assert got(res) == e
        assert res[1].path & T.PATH_OTHER
        e20 = expected(paths, QDENSE, 20)
        assert got(eng.search(blocks, T.Pipeline(request(QDENSE)), limit=20)) == e20
    finally:
        for b in blocks:
            b.close()
        eng.close()


def test_devices_serve_concurrent_callers(paths):
    """Two threads, each searching blocks spread over both contexts at once."""
    import threading
    eng = T.Engine(devices=[0, 0])
    blocks = [eng.open_block(p, device=i % 2) for i, p in enumerate(paths)]
    pl = {0: T.Pipeline(request(QA)), 1: T.Pipeline(request(QB))}
    exp = {0: expected(paths, QA), 1: expected(paths, QB)}
    errors = []

    def worker(t):
        try:
            for r in range(8):
                k = (t + r) % 2
                assert got(eng.search(blocks, pl[k])) == exp[k], (t, r)
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        assert not errors, errors[0]
    finally:
        for b in blocks:
            b.close()
        eng.close()


_CHILD = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
import tempo_amd as T
eng = T.Engine(devices=[0])
print("ready", flush=True)
sys.stdin.readline()  # (holds its context until the parent writes a line)
eng.close()
print("closed", flush=True)
"""


def test_another_process_on_the_gpu(engine, paths, tmp_path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    blocks = [engine.open_block(p) for p in paths[:3]]
    pa = T.Pipeline(request(QA))
    e = expected(paths[:3], QA)
    child = None
    try:
        res = engine.search(blocks, pa)
        assert got(res) == e and res[1].path == T.PATH_RESIDENT
        c0 = engine.resident_counters()
        child = subprocess.Popen([sys.executable, "-c", _CHILD, root], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 text=True)
        line = child.stdout.readline()
        assert line.strip() == "ready", line
        for _ in range(3):
            res = engine.search(blocks, pa)
            assert got(res) == e
            assert res[1].path == T.PATH_PLAIN | T.PATH_COTENANT, res[1].path
        c1 = engine.resident_counters()
        assert c1["cotenant_queries"] - c0["cotenant_queries"] == 3 and c1["queries"] == c0["queries"], (c0, c1)
        child.stdin.write("\n")
        child.stdin.flush()
        assert child.stdout.readline().strip() == "closed"
        assert child.wait(60) == 0
        child = None
        res = engine.search(blocks, pa)
        assert got(res) == e and res[1].path == T.PATH_RESIDENT  # (alone again)
    finally:
        if child is not None:
            child.kill()
            child.wait(30)
        for b in blocks:
            b.close()
