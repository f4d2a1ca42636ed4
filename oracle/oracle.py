"""ctypes binding of the CPU ORACLE (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, where it is the checker / the baseline, never the
thing measured as the product. See tsg_oracle.h for what it restates and how
it is pinned.
"""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORACLE_LIB_PATH") or os.path.join(HERE, "build", "liboracle.so")  # (override: the ASan build, tests/sanitize)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class Request(C.Structure):
    _fields_ = [("ntags", C.c_uint32),
                ("tag_keys", C.POINTER(C.c_char_p)), ("tag_key_lens", C.POINTER(C.c_uint32)),
                ("tag_values", C.POINTER(C.c_char_p)), ("tag_value_lens", C.POINTER(C.c_uint32)),
                ("min_duration_ms", C.c_uint32), ("max_duration_ms", C.c_uint32),
                ("limit", C.c_uint32), ("start", C.c_uint32), ("end", C.c_uint32)]


class Match(C.Structure):
    _fields_ = [("id", C.c_uint8 * 16), ("id_len", C.c_uint32), ("block_idx", C.c_uint32),
                ("entry_idx", C.c_uint64), ("start_ns", C.c_uint64), ("end_ns", C.c_uint64),
                ("duration_ms", C.c_uint32), ("svc_off", C.c_uint32), ("svc_len", C.c_uint32),
                ("name_off", C.c_uint32), ("name_len", C.c_uint32)]


class Metrics(C.Structure):
    _fields_ = [("traces_inspected", C.c_uint32), ("blocks_inspected", C.c_uint32),
                ("blocks_skipped", C.c_uint32), ("pad", C.c_uint32), ("bytes_inspected", C.c_uint64)]


class Result(C.Structure):
    _fields_ = [("n", C.c_uint64), ("m", C.POINTER(Match)), ("strings", C.POINTER(C.c_char)),
                ("strings_len", C.c_uint64), ("metrics", Metrics), ("status", C.c_int32), ("pad", C.c_int32),
                ("nblocks", C.c_uint64), ("block_status", C.POINTER(C.c_int32))]


class Hit(C.Structure):
    _fields_ = [("id_idx", C.c_uint32), ("block_idx", C.c_uint32), ("record_idx", C.c_int32),
                ("record_length", C.c_uint32), ("record_start", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.orc_block_load.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.orc_block_set_pages.argtypes = [vp, C.c_uint32, C.c_uint32]
        L.orc_block_set_pages.restype = None
        L.orc_wal_block_load.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.orc_entry_to_bytes.argtypes = [C.c_char_p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint32,
                                         C.POINTER(C.c_char_p), C.POINTER(C.c_uint32), C.POINTER(C.c_char_p),
                                         C.POINTER(C.c_uint32), C.POINTER(C.POINTER(C.c_uint8)),
                                         C.POINTER(C.c_size_t)]
        L.orc_block_free.argtypes = [vp]
        L.orc_block_bytes.argtypes = [vp]
        L.orc_block_bytes.restype = C.c_uint64
        L.orc_search_seeded.argtypes = [C.POINTER(vp), C.c_uint32, C.POINTER(Request), C.c_uint32, C.c_void_p,
                                        C.c_uint64, C.POINTER(C.POINTER(Result))]
        L.orc_search.argtypes = [C.POINTER(vp), C.c_uint32, C.POINTER(Request), C.c_uint32, C.c_int,
                                 C.POINTER(C.POINTER(Result))]
        L.orc_combine.argtypes = [C.POINTER(Result), C.c_uint32, C.POINTER(C.POINTER(Result))]
        L.orc_result_free.argtypes = [C.POINTER(Result)]
        L.orc_pipeline_matches_entry.argtypes = [C.POINTER(Request), C.c_char_p, C.c_size_t]
        L.orc_pipeline_matches_block.argtypes = [C.POINTER(Request), C.c_char_p, C.c_size_t]
        L.orc_contains_tag_entry.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                             C.c_size_t]
        L.orc_xxhash64.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_xxhash64.restype = C.c_uint64
        L.orc_fnv1_32.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_fnv1_32.restype = C.c_uint32
        L.orc_crc32c.argtypes = [C.c_char_p, C.c_size_t]
        L.orc_crc32c.restype = C.c_uint32
        L.orc_murmur3_128.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint64)]
        L.orc_snappy_framed_decode.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(C.c_uint8)),
                                               C.POINTER(C.c_size_t)]
        L.orc_free.argtypes = [vp]
        L.orc_v2block_load.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.orc_v2block_free.argtypes = [vp]
        L.orc_v2_bloom_test.argtypes = [vp, C.c_char_p, C.c_size_t]
        L.orc_v2_index_find.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_int64),
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        L.orc_v2_find.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(C.c_uint8)),
                                  C.POINTER(C.c_size_t)]
        L.orc_v2_include_block.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_uint32, C.c_char_p, C.c_char_p]
        L.orc_lookup_ids.argtypes = [C.POINTER(vp), C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                     C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.POINTER(Hit)),
                                     C.POINTER(C.c_uint64)]
        L.orc_colblock_build.argtypes = [vp, C.POINTER(vp)]
        L.orc_colblock_free.argtypes = [vp]
        L.orc_colblock_entries.argtypes = [vp]
        L.orc_colblock_entries.restype = C.c_uint64
        L.orc_columnar_search.argtypes = [C.POINTER(vp), C.c_uint32, C.POINTER(Request), C.c_int,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_live_block_load_mem.argtypes = [C.c_char_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                              C.POINTER(vp)]
        pp = C.POINTER(C.POINTER(C.c_uint8))
        sz = C.POINTER(C.c_size_t)
        L.orc_block_tags.argtypes = [vp, pp, sz, sz]
        L.orc_block_tag_values.argtypes = [vp, C.c_char_p, C.c_size_t, pp, sz, sz]
        L.orc_search_tags.argtypes = [C.POINTER(vp), C.c_uint32, pp, sz, sz]
        L.orc_search_tag_values.argtypes = [C.POINTER(vp), C.c_uint32, C.c_char_p, C.c_size_t, C.c_int64, pp, sz, sz]
        L.orc_v2_shard_count.argtypes = [vp]
        L.orc_v2_shard_count.restype = C.c_uint32
        _lib = L
    return _lib


def make_request(tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=0):
    """tempopb.SearchRequest -> orc_request (keeps the byte buffers alive)."""
    tags = dict(tags or {})
    ks = [k.encode() if isinstance(k, str) else k for k in tags.keys()]
    vs = [v.encode() if isinstance(v, str) else v for v in tags.values()]
    n = len(ks)
    r = Request()
    r.ntags = n
    r._k = (C.c_char_p * max(n, 1))(*ks)
    r._v = (C.c_char_p * max(n, 1))(*vs)
    r._kl = (C.c_uint32 * max(n, 1))(*[len(k) for k in ks])
    r._vl = (C.c_uint32 * max(n, 1))(*[len(v) for v in vs])
    r.tag_keys, r.tag_values = r._k, r._v
    r.tag_key_lens, r.tag_value_lens = r._kl, r._vl
    r.min_duration_ms, r.max_duration_ms, r.start, r.end, r.limit = min_ms, max_ms, start, end, limit
    return r


class Block:
    def __init__(self, path, wal=False, pages=None):
        """pages = (first_page, npages): only those index records are searched (npages 0 = to
        the end); a range after page 0 counts neither the header nor the block itself."""
        self.h = C.c_void_p()
        load = lib().orc_wal_block_load if wal else lib().orc_block_load
        rc = load(path.encode(), C.byref(self.h))
        if rc != 0:
            raise OSError(f"orc_{'wal_' if wal else ''}block_load({path}) -> {rc}")
        if pages is not None:
            lib().orc_block_set_pages(self.h, int(pages[0]), int(pages[1]))

    def nbytes(self):
        return lib().orc_block_bytes(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_block_free(self.h)
            self.h = None


def live_wire(traces):
    """[[segment bytes, ...] per trace] -> (bytes, seg_off u64[nsegs+1], trace_seg u64[ntraces+1])."""
    import numpy as np
    segs = [s for t in traces for s in t]
    seg_off = np.zeros(len(segs) + 1, dtype=np.uint64)
    if segs:
        seg_off[1:] = np.cumsum([len(s) for s in segs])
    trace_seg = np.zeros(len(traces) + 1, dtype=np.uint64)
    if traces:
        trace_seg[1:] = np.cumsum([len(t) for t in traces])
    return b"".join(segs), seg_off, trace_seg


class LiveBlock:
    """Live traces (instance.searchLiveTraces): traces = [[segment, ...], ...] in the
    ingester's iteration order; each segment a SearchEntry flatbuffer."""

    def __init__(self, traces):
        data, seg_off, trace_seg = live_wire(traces)
        self._keep = (data, seg_off, trace_seg)
        self.h = C.c_void_p()
        rc = lib().orc_live_block_load_mem(data, seg_off.ctypes.data, len(seg_off) - 1, trace_seg.ctypes.data,
                                           len(trace_seg) - 1, C.byref(self.h))
        if rc != 0:
            raise OSError(f"orc_live_block_load_mem -> {rc}")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_block_free(self.h)
            self.h = None


def _strings(fn, *args):
    out, ln, n = C.POINTER(C.c_uint8)(), C.c_size_t(), C.c_size_t()
    rc = fn(*args, C.byref(out), C.byref(ln), C.byref(n))
    if rc != 0:
        return rc, None
    b = C.string_at(out, ln.value) if ln.value else b""
    lib().orc_free(out)
    res, o = [], 0
    for _ in range(n.value):
        k = int.from_bytes(b[o:o + 4], "little")
        res.append(b[o + 4:o + 4 + k])
        o += 4 + k
    return 0, res


def block_tags(block):
    """(status, sorted tag names) of one block (oracle)."""
    return _strings(lib().orc_block_tags, block.h)


def block_tag_values(block, key):
    key = key.encode() if isinstance(key, str) else key
    return _strings(lib().orc_block_tag_values, block.h, key, len(key))


def search_tags(blocks):
    """instance.SearchTags over blocks (live blocks first): (status, sorted names)."""
    arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
    return _strings(lib().orc_search_tags, arr, len(blocks))


def search_tag_values(blocks, key, max_bytes=-1):
    """instance.SearchTagValues over blocks (live first, MapSizeWithinLimit checks)."""
    key = key.encode() if isinstance(key, str) else key
    arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
    return _strings(lib().orc_search_tag_values, arr, len(blocks), key, len(key), max_bytes)


def _unpack(res):
    r = res.contents
    strings = C.string_at(r.strings, r.strings_len) if r.strings_len else b""
    out = []
    for i in range(r.n):
        m = r.m[i]
        out.append({
            "id": bytes(m.id), "id_len": m.id_len, "block_idx": m.block_idx, "entry_idx": m.entry_idx,
            "start_ns": m.start_ns, "end_ns": m.end_ns, "duration_ms": m.duration_ms,
            "root_service": strings[m.svc_off:m.svc_off + m.svc_len],
            "root_name": strings[m.name_off:m.name_off + m.name_len],
        })
    met = {"traces_inspected": r.metrics.traces_inspected, "blocks_inspected": r.metrics.blocks_inspected,
           "blocks_skipped": r.metrics.blocks_skipped, "bytes_inspected": r.metrics.bytes_inspected,
           "block_status": [r.block_status[i] for i in range(r.nblocks)]}
    return out, met, r.status


def search(blocks, tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=0, nthreads=1, combine=None, seen=None):
    """BackendSearchBlock.Search over blocks (oracle). Returns (matches, metrics, status).
    seen: trace IDs ((n, 16) uint8) a consumer took before these blocks (orc_search_seeded)."""
    req = make_request(tags, min_ms, max_ms, start, end, limit)
    arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
    res = C.POINTER(Result)()
    if seen is not None and len(seen):
        import numpy as np
        sa = np.ascontiguousarray(seen, dtype=np.uint8).reshape(-1, 16)
        lib().orc_search_seeded(arr, len(blocks), C.byref(req), limit, sa.ctypes.data, sa.shape[0], C.byref(res))
    else:
        lib().orc_search(arr, len(blocks), C.byref(req), limit, nthreads, C.byref(res))
    try:
        if combine is not None:
            fin = C.POINTER(Result)()
            lib().orc_combine(res, combine, C.byref(fin))
            try:
                return _unpack(fin)
            finally:
                lib().orc_result_free(fin)
        return _unpack(res)
    finally:
        lib().orc_result_free(res)


class V2Block:
    def __init__(self, path):
        self.h = C.c_void_p()
        rc = lib().orc_v2block_load(path.encode(), C.byref(self.h))
        if rc != 0:
            raise OSError(f"orc_v2block_load({path}) -> {rc}")

    def bloom_test(self, tid):
        return lib().orc_v2_bloom_test(self.h, tid, len(tid))

    def index_find(self, tid):
        i, s, l = C.c_int64(), C.c_uint64(), C.c_uint32()
        rc = lib().orc_v2_index_find(self.h, tid, len(tid), C.byref(i), C.byref(s), C.byref(l))
        assert rc == 0, rc
        return i.value, s.value, l.value

    def find(self, tid):
        p, n = C.POINTER(C.c_uint8)(), C.c_size_t()
        rc = lib().orc_v2_find(self.h, tid, len(tid), C.byref(p), C.byref(n))
        assert rc == 0, rc
        if not p:
            return None
        b = C.string_at(p, n.value)
        lib().orc_free(p)
        return b

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_v2block_free(self.h)
            self.h = None


def lookup(blocks, ids, ts=0, te=0, bstart=None, bend=None, nthreads=1):
    """Batched lookup (oracle): list of (id_idx, block_idx, record_idx, start, length)."""
    import numpy as np
    ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 16)
    arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
    hp, n = C.POINTER(Hit)(), C.c_uint64()
    rc = lib().orc_lookup_ids(arr, len(blocks), ids.ctypes.data, ids.shape[0], ts, te, bstart, bend, nthreads,
                              C.byref(hp), C.byref(n))
    out = [(hp[i].id_idx, hp[i].block_idx, hp[i].record_idx, hp[i].record_start, hp[i].record_length)
           for i in range(n.value)]
    lib().orc_free(hp)
    return rc, out


def entry_to_bytes(entry):
    """SearchEntryMutable.ToBytes of {"id", "start", "end", "tags": {k: [v]}} (oracle builder)."""
    pairs = []
    for k, vs in entry.get("tags", {}).items():
        for v in ([vs] if isinstance(vs, (str, bytes)) else vs):
            pairs.append((k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str) else v))
    n = len(pairs)
    K = (C.c_char_p * max(n, 1))(*[k for k, _ in pairs])
    V = (C.c_char_p * max(n, 1))(*[v for _, v in pairs])
    KL = (C.c_uint32 * max(n, 1))(*[len(k) for k, _ in pairs])
    VL = (C.c_uint32 * max(n, 1))(*[len(v) for _, v in pairs])
    out, ol = C.POINTER(C.c_uint8)(), C.c_size_t()
    tid = entry["id"]
    lib().orc_entry_to_bytes(tid, len(tid), entry.get("start", 0), entry.get("end", 0), n, K, KL, V, VL,
                             C.byref(out), C.byref(ol))
    b = C.string_at(out, ol.value)
    lib().orc_free(out)
    return b


def snappy_framed_decode(b):
    """The C oracle's snappy framing-format decoder (golang/snappy Reader restated)."""
    out, n = C.POINTER(C.c_uint8)(), C.c_size_t()
    rc = lib().orc_snappy_framed_decode(b, len(b), C.byref(out), C.byref(n))
    if rc != 0:
        raise ValueError("snappy decode failed (%d)" % rc)
    r = C.string_at(out, n.value)
    lib().orc_free(out)
    return r


def xxhash64(b):
    return lib().orc_xxhash64(b, len(b))


def fnv1_32(b):
    return lib().orc_fnv1_32(b, len(b))


def crc32c(b):
    return lib().orc_crc32c(b, len(b))


def murmur3_128(b):
    out = (C.c_uint64 * 2)()
    lib().orc_murmur3_128(b, len(b), out)
    return out[0], out[1]


def contains_tag_entry(fb, k, v):
    return bool(lib().orc_contains_tag_entry(fb, len(fb), k, len(k), v, len(v)))


def pipeline_matches_entry(fb, **req):
    r = make_request(**req)
    return bool(lib().orc_pipeline_matches_entry(C.byref(r), fb, len(fb)))


def pipeline_matches_block(fb, **req):
    r = make_request(**req)
    return bool(lib().orc_pipeline_matches_block(C.byref(r), fb, len(fb)))


class ColumnarBlock:
    """CPU columnar baseline: a backend search block decoded once into host columns
    (orc_colblock_build); searched by columnar_search over nthreads threads."""

    def __init__(self, block):
        self.h = C.c_void_p()
        rc = lib().orc_colblock_build(block.h, C.byref(self.h))
        if rc != 0:
            raise OSError(f"orc_colblock_build -> {rc}")

    def entries(self):
        return lib().orc_colblock_entries(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_colblock_free(self.h)
            self.h = None


def columnar_search(cblocks, tags=None, min_ms=0, max_ms=0, start=0, end=0, nthreads=1):
    """(match count, order-independent hash of the (block, scan position) matches)."""
    req = make_request(tags, min_ms, max_ms, start, end)
    arr = (C.c_void_p * max(len(cblocks), 1))(*[b.h for b in cblocks])
    m, h = C.c_uint64(), C.c_uint64()
    lib().orc_columnar_search(arr, len(cblocks), C.byref(req), nthreads, C.byref(m), C.byref(h))
    return m.value, h.value


def match_hash(matches):
    """The columnar_search hash of a match list [(block_idx, entry_idx), ...]."""
    return sum(((b << 32) | e) * 0x9E3779B97F4A7C15 for b, e in matches) % (1 << 64)
