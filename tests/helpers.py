"""Shared test helpers: synthetic entries, block writing, oracle/engine comparison."""
import os
import random
import tempfile

from oracle import oracle as O
import tempo_amd as T


def ref_id(i, n=16):
    """binary.LittleEndian.PutUint32(id, uint32(i)) into an n-byte buffer
    (tempodb/search/backend_search_block_test.go:63-64)."""
    return i.to_bytes(4, "little") + bytes(n - 4)


def gen_search_data(i):
    """genSearchData (backend_search_block_test.go:24-31)."""
    return {"key%d" % i: ["value_A_%d" % i, "value_B_%d" % i]}


def write_block(tmpdir, name, entries, enc=T.ENC_SNAPPY, page_size=0):
    path = os.path.join(tmpdir, name)
    T.write_search_block(path, entries, enc, page_size)
    return path


def random_entries(rng, n, nkeys=6, nvals=5, multi=3, id_len=16, with_names=True, t0=1_700_000_000 * 10**9,
                   zero_end_frac=0.02):
    ents = []
    ids = set()
    while len(ids) < n:
        ids.add(bytes(rng.getrandbits(8) for _ in range(id_len)))
    for tid in sorted(ids):
        tags = {}
        for k in range(nkeys):
            if rng.random() < 0.8:
                vals = sorted({"v%d-%s" % (rng.randrange(nvals), "xyz"[rng.randrange(3)])
                               for _ in range(1 + rng.randrange(multi))})
                tags["k%d" % k] = vals
        if with_names:
            tags["root.service.name"] = ["svc-%d" % rng.randrange(4)]
            tags["root.name"] = ["op-%d" % rng.randrange(7)]
        start = t0 + rng.randrange(3600 * 10**9)
        dur = int(rng.lognormvariate(17.7, 1.5))
        end = start + dur
        if rng.random() < zero_end_frac:
            end = 0
        ents.append({"id": tid, "start": start, "end": end, "tags": tags})
    return ents


def match_key(m):
    """Comparable tuple for an oracle match dict."""
    return (m["block_idx"], m["entry_idx"], m["id"], m["start_ns"], m["end_ns"], m["duration_ms"],
            m["root_service"], m["root_name"])


def tsg_key(m):
    return (m.block_idx, m.entry_idx, m.trace_id, m.start_time_unix_nano, m.end_time_unix_nano, m.duration_ms,
            m.root_service_name.encode(), m.root_trace_name.encode())
