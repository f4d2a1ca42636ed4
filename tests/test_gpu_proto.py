"""GPU parity for the proto-object backend search:
tsg_proto_search (loader + proto_scan_kernel + the host replay of BackendBlock.Search)
against the oracle (oracle/proto_oracle.py, pinned by tests/test_proto_oracle.py).

Every comparison covers the full ordered result (trace id, root service / span name,
start ns, DurationMs, object position) and the three SearchMetrics, or that both raise.
Blocks: synthetic v1 and v2 blocks (none / snappy pages, small pages so the paged
iterator chunks and the partial page ranges matter, corrupt objects for the error
path) and the reference's tempo-cli block (zstd, dataEncoding v1, 621 real traces,
cmd/tempo-cli/test-data, copied under tests/golden/tempo_cli).
"""
import os
import random

import numpy as np
import pytest

from oracle import proto_oracle as P
import tempo_amd as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SEC = 1_000_000_000
T0 = 1_700_000_000

SVCS = ["frontend", "cart", "checkout", "payment", "db-proxy"]
OPS = ["GET /api", "POST /cart", "SELECT", "charge", "render", "op-%d"]
URLS = ["/api/v1/users/%d", "/cart/%d/items", "/static/app.js"]


def rand_trace(rng, ti):
    """A random trace (batches of spans): string/int/double/bool attributes, roots or not."""
    base = T0 + rng.randrange(0, 3600)
    batches = []
    for b in range(rng.randint(1, 3)):
        res = {"service.name": rng.choice(SVCS)} if rng.random() > 0.05 else None
        if res is not None and rng.random() < 0.3:
            res["cluster"] = rng.choice(["prod", "dev", "staging"])
        if res is not None and rng.random() < 0.1:
            res["service.name"] = rng.choice([7, True, 2.5])  # non-string service.name
        spans = []
        for s in range(rng.randint(0, 4)):
            st = base * SEC + rng.randrange(0, 5000) * 1_000_000 + rng.randrange(0, 999_999)
            sp = {"name": rng.choice(OPS) if rng.random() > 0.1 else "op-%d" % rng.randrange(20),
                  "start": st, "end": st + rng.randrange(0, 30_000) * 1_000_000 + rng.randrange(0, 999_999),
                  "parent": b"" if (s == 0 and b == 0 and rng.random() > 0.2) else bytes([1 + rng.randrange(200)]) * 8,
                  "code": rng.choice([0, 1, 2, None]), "attrs": {}}
            if rng.random() < 0.6:
                u = rng.choice(URLS)
                sp["attrs"]["http.url"] = u % rng.randrange(100) if "%" in u else u
            if rng.random() < 0.5:
                sp["attrs"]["http.status_code"] = rng.choice([200, 201, 404, 500, -1, 2 ** 40])
            if rng.random() < 0.3:
                sp["attrs"]["ratio"] = rng.choice([0.5, 42.42, 1e-3, -0.0, 1e300, float(rng.randrange(10))])
            if rng.random() < 0.3:
                sp["attrs"]["error"] = rng.choice([True, False])
            if rng.random() < 0.2:
                sp["attrs"]["name"] = rng.choice(["cart-item", "test"])
            if rng.random() < 0.1:
                sp["attrs"]["tags"] = ["a", 1]  # array value: never matches
            spans.append(sp)
        batches.append({"resource": res, "spans": spans})
    return batches, base


def make_block(path, rng, n, v2, encoding, downsample=4096, corrupt=()):
    ids = sorted({bytes(rng.randrange(256) for _ in range(16)) for _ in range(n)})
    objs = []
    for i, _ in enumerate(ids):
        batches, base = rand_trace(rng, i)
        obj = P.enc_object(batches, v2, base, base + rng.randrange(0, 40), split=rng.choice([1, 1, 2]))
        if i in corrupt:
            obj = obj[:8] + b"\x0a\xff\xff" if v2 else b"\x0a\xff\xff"  # truncated length-delimited field
        objs.append(obj)
    T.write_v2_block(path, np.frombuffer(b"".join(ids), dtype=np.uint8).reshape(-1, 16), objs,
                     encoding=encoding, data_encoding="v2" if v2 else "v1", index_downsample_bytes=downsample)
    return ids


def key(r):
    return [(t.trace_id, t.root_service_name.encode("utf-8", "surrogateescape"),
             t.root_trace_name.encode("utf-8", "surrogateescape"), t.start_time_unix_nano, t.duration_ms, o)
            for t, o in zip(r.traces, r.object_idx)], (r.inspected_traces, r.inspected_bytes, r.skipped_traces)


def okey(res):
    traces, met = res
    return [(t["trace_id"], t["root_service_name"], t["root_trace_name"], t["start_time_unix_nano"],
             t["duration_ms"], t["object_idx"]) for t in traces], \
        (met["inspected_traces"], met["inspected_bytes"], met["skipped_traces"])


def check(engine, blk, ob, **req):
    try:
        exp = okey(ob.search(**req))
    except P.ProtoError:
        exp = "error"
    try:
        got = key(engine.proto_search(blk, **req))
    except T.TsgError as e:
        assert e.code == T.TSG_E_CORRUPT, e
        got = "error"
    assert got == exp, req
    return got


def queries(rng):
    yield dict(start=0, end=2 ** 32 - 1, limit=1000)
    yield dict(start=T0 + 900, end=T0 + 2700, limit=20)
    yield dict(start=0, end=2 ** 32 - 1, limit=0)  # Search breaks after the first object
    yield dict(start=0, end=0, limit=50)            # End 0: the reference compares it too
    for _ in range(40):
        tags = {}
        for _ in range(rng.choice([0, 1, 1, 2, 3])):
            k = rng.choice(["service.name", "cluster", "http.url", "http.status_code", "ratio", "error", "name",
                            "status.code", "missing.key", "tags"])
            v = {"service.name": rng.choice(["cart", "pay", "front", "svc", ""]),
                 "cluster": rng.choice(["prod", "dev", "o"]),
                 "http.url": rng.choice(["/api", "users/1", "items", "/static/app.js"]),
                 "http.status_code": rng.choice(["200", "404", "500", "-1", "1099511627776", "abc", "2e2"]),
                 "ratio": rng.choice(["0.5", "42.42", "1e-3", "-0", "0", "1e300", "nan", "0x1p-1"]),
                 "error": rng.choice(["true", "false", "True", "1"]),
                 "name": rng.choice(["GET /api", "SELECT", "op-3", "test", "cart-item", "GET"]),
                 "status.code": rng.choice(["ok", "error", "unset", "bogus"]),
                 "missing.key": "x", "tags": "a"}[k]
            tags[k] = v
        s = T0 + rng.randrange(0, 3600)
        yield dict(tags=tags, start=rng.choice([0, s]), end=rng.choice([s + rng.randrange(0, 7200), 2 ** 32 - 1]),
                   min_ms=rng.choice([0, 0, 1000, 5000]), max_ms=rng.choice([0, 0, 2000, 20000]),
                   limit=rng.choice([1, 5, 20, 1000]), max_bytes=rng.choice([0, 0, 600]),
                   **rng.choice([{}, {}, dict(start_page=rng.randrange(4), total_pages=rng.randrange(1, 4))]),
                   chunk_size_bytes=rng.choice([1_000_000, 10_000]))


@pytest.mark.parametrize("v2,encoding", [(True, T.ENC_NONE), (True, T.ENC_SNAPPY), (False, T.ENC_SNAPPY)],
                         ids=["v2-none", "v2-snappy", "v1-snappy"])
def test_proto_search_synthetic(engine, tmp_path, v2, encoding):
    rng = random.Random(11 + v2 + 3 * encoding)
    path = os.path.join(str(tmp_path), "pb")
    make_block(path, rng, 400, v2, encoding)
    blk = engine.open_proto_block(path)
    ob = P.ProtoBlock(path)
    info = blk.info()
    assert info["objects"] == 400 and info["pages"] > 4
    n_match = 0
    for q in queries(rng):
        got = check(engine, blk, ob, **q)
        n_match += len(got[0]) if got != "error" else 0
    assert n_match > 100
    blk.close()


@pytest.mark.parametrize("v2", [True, False], ids=["v2", "v1"])
def test_proto_search_errors(engine, tmp_path, v2):
    """Objects that fail to decode: an error exactly when Search reaches them before its
    limit break (v2: only if they pass the FastRange/duration prefilter)."""
    rng = random.Random(5 + v2)
    path = os.path.join(str(tmp_path), "pe")
    make_block(path, rng, 200, v2, T.ENC_NONE, corrupt=(37, 150))
    blk = engine.open_proto_block(path)
    ob = P.ProtoBlock(path)
    outcomes = set()
    for lim in (1, 5, 20, 30, 1000):
        for q in (dict(start=0, end=2 ** 32 - 1), dict(start=T0 + 100, end=T0 + 200),
                  dict(tags={"service.name": "cart"}, start=0, end=2 ** 32 - 1)):
            got = check(engine, blk, ob, limit=lim, **q)
            outcomes.add(got == "error")
    assert outcomes == {True, False}


def test_proto_search_tempo_cli_block(engine):
    """The reference's tempo-cli test block: zstd pages, dataEncoding v1, real traces."""
    path = os.path.join(GOLD, "tempo_cli")
    blk = engine.open_proto_block(path)
    ob = P.ProtoBlock(path)
    assert blk.info()["objects"] == 621
    full = check(engine, blk, ob, start=0, end=2 ** 32 - 1, limit=1000)
    assert len(full[0]) == 621
    traces = [t for t in full[0]]
    rng = random.Random(3)
    svcs = sorted({t[1].decode() for t in traces if t[1]})
    names = sorted({t[2].decode() for t in traces})
    for _ in range(30):
        tags = {}
        if rng.random() < 0.7:
            tags["service.name"] = rng.choice(svcs)[: rng.randint(1, 6)]
        if rng.random() < 0.4:
            tags["name"] = rng.choice(names)
        if rng.random() < 0.3:
            tags[rng.choice(["status.code", "error"])] = rng.choice(["ok", "error", "unset", "true"])
        check(engine, blk, ob, tags=tags, start=0, end=2 ** 32 - 1, min_ms=rng.choice([0, 10, 100]),
              max_ms=rng.choice([0, 1000]), limit=rng.choice([1, 20, 1000]))
    blk.close()
