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


# ---- damaged blocks (BackendSearchBlock.Search's error paths) ------------------------
def _meta(path):
    import json
    with open(os.path.join(path, "search.meta.json")) as f:
        return json.load(f)


def _write_meta(path, meta):
    import json
    with open(os.path.join(path, "search.meta.json"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")))


def index_records(path):
    """The (id, start, length) records of a block's search-index (v2 index pages)."""
    import struct
    meta = _meta(path)
    ps, n = meta["indexPageSize"], meta["indexRecords"]
    rpp = (ps - 14) // 28
    raw = open(os.path.join(path, "search-index"), "rb").read()
    out = []
    for i in range(n):
        p, r = divmod(i, rpp)
        rec = raw[p * ps + 14 + 28 * r: p * ps + 14 + 28 * (r + 1)]
        out.append((rec[:16],) + struct.unpack("<QI", rec[16:]))
    return out


def repage_index(path, rpp):
    """Rewrite search-index with `rpp` records per page (indexPageSize = 14 + 28 rpp, a
    value the reference reads from search.meta.json), so a test can damage page k > 0."""
    import struct
    recs = index_records(path)
    ps = 14 + 28 * rpp
    out = bytearray()
    for p0 in range(0, len(recs), rpp):
        data = b"".join(i + struct.pack("<QI", s, l) for i, s, l in recs[p0:p0 + rpp])
        data += bytes(28 * rpp - len(data))
        out += struct.pack("<IHQ", ps, 8, O.xxhash64(data)) + data
    open(os.path.join(path, "search-index"), "wb").write(bytes(out))
    meta = _meta(path)
    meta["indexPageSize"] = ps
    _write_meta(path, meta)


def damage_index_page_checksum(path, page):
    """Flip a byte of index page `page`'s data: getPage fails its checksum."""
    ps = _meta(path)["indexPageSize"]
    p = os.path.join(path, "search-index")
    b = bytearray(open(p, "rb").read())
    b[page * ps + 14 + 3] ^= 0x5A
    open(p, "wb").write(bytes(b))


def zero_index_record(path, k):
    """Zero record k and re-checksum its page: At(k) fails ('unexpected zero value record')."""
    import struct
    meta = _meta(path)
    ps = meta["indexPageSize"]
    rpp = (ps - 14) // 28
    pg, r = divmod(k, rpp)
    p = os.path.join(path, "search-index")
    b = bytearray(open(p, "rb").read())
    o = pg * ps + 14
    b[o + 28 * r: o + 28 * (r + 1)] = bytes(28)
    b[pg * ps + 6: pg * ps + 14] = struct.pack("<Q", O.xxhash64(bytes(b[o:pg * ps + ps])))
    open(p, "wb").write(bytes(b))


def damage_data_page(path, k, how="payload"):
    """Damage data page k of the `search` file. payload: flip a byte in the middle of the
    (compressed) page payload; length: break the page's totalLength field; truncate: cut
    the file inside page k (its ReadAt fails)."""
    import struct
    _, start, length = index_records(path)[k]
    p = os.path.join(path, "search")
    b = bytearray(open(p, "rb").read())
    if how == "payload":
        b[start + 6 + (length - 6) // 2] ^= 0xA5
    elif how == "length":
        b[start:start + 4] = struct.pack("<I", length + 1)
    elif how == "objlen":  # (encoding none) the object's total length past the page
        b[start + 6:start + 10] = struct.pack("<I", 0x7FFFFFF0)
    elif how == "truncate":
        b = b[:start + length // 2]
    open(p, "wb").write(bytes(b))


def shim_digest(per_block):
    """tsgx_shim_pattern's per-round digest (shim_pattern.cpp result_digest) from the oracle's
    ordered matches of each block of the set: the sum mod 2^64 over blocks i of FNV-1a 64 over
    (i as u32, then per match its scan position u64, its id right-aligned in 16 bytes, its start u64)."""
    import struct
    M = (1 << 64) - 1
    total = 0
    for i, matches in enumerate(per_block):
        h = 0xcbf29ce484222325
        buf = bytearray(struct.pack("<I", i))
        for m in matches:
            buf += struct.pack("<Q", m["entry_idx"]) + bytes(16 - len(m["id"])) + m["id"] + struct.pack("<Q", m["start_ns"])
        for b in buf:
            h = ((h ^ b) * 0x100000001b3) & M
        total = (total + h) & M
    return total
