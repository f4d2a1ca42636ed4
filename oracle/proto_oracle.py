"""Proto-object backend search oracle (test infrastructure only — never imported by the
product path): a pure-Python restatement of

  v2.BackendBlock.Search      tempodb/encoding/v2/backend_block.go:159-231
  pagedIterator.Next          tempodb/encoding/v2/iterator_paged.go:62-131 (chunked page reads)
  indexReader.At / getPage    tempodb/encoding/v2/index_reader.go:42-82,116-143
  dataReader.Read             tempodb/encoding/v2/data_reader.go:45-125 (page framing, decompress)
  UnmarshalAndAdvanceBuffer   tempodb/encoding/v2/object.go:82-113
  ObjectDecoder v1 / v2       pkg/model/v1/object_decoder.go, pkg/model/v2/object_decoder.go:28-134,
                              pkg/model/v2/segment_decoder.go:106-122
  gogo Unmarshal              pkg/tempopb/{tempo,trace/v1/trace,common/v1/common,resource/v1/resource}.pb.go
  MatchesProto                pkg/model/trace/matches.go:33-184
  strconv.ParseInt/Float/Bool (Go standard library, decimal/hex float literal grammar)

Pinned by tests/test_proto_oracle.py against the reference's TestMatches table
(pkg/model/object_decoder_test.go:49-478, both encodings) and TestMatchesFails.
Where the reference panics (nil AnyValue, nil Status under an error/status.code tag,
nil Resource on the root span's batch) the value is taken as absent / UNSET / no
resource attributes, as the engine does.
Page decompression uses independent codecs: none, snappy (the C oracle's framed
decoder) and zstd (pyarrow = libzstd).
"""
import json
import math
import os
import re
import struct

ROOT_NOT_YET = "<root span not yet received>"


class ProtoError(Exception):
    pass


# ---- protobuf wire format (gogo semantics) ------------------------------------------
def _varint(b, i):
    v = 0
    shift = 0
    while True:
        if shift >= 64:
            raise ProtoError("integer overflow")
        if i >= len(b):
            raise ProtoError("unexpected EOF")
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v & 0xFFFFFFFFFFFFFFFF, i
        shift += 7


def _skip(b, i, wt, depth=0):
    if wt == 0:
        return _varint(b, i)[1]
    if wt == 1:
        if len(b) - i < 8:
            raise ProtoError("EOF")
        return i + 8
    if wt == 2:
        n, i = _varint(b, i)
        if n > len(b) - i:
            raise ProtoError("EOF")
        return i + n
    if wt == 5:
        if len(b) - i < 4:
            raise ProtoError("EOF")
        return i + 4
    if wt == 3:
        if depth > 64:
            raise ProtoError("depth")
        while True:
            tag, i = _varint(b, i)
            w = tag & 7
            if w == 4:
                return i
            if tag >> 3 == 0:
                raise ProtoError("illegal tag 0")
            i = _skip(b, i, w, depth + 1)
    raise ProtoError("illegal wireType %d" % wt)


def fields(b):
    """(field, wiretype, value, raw): value = int (0/1/5) or bytes (2); unknown fields too."""
    i = 0
    while i < len(b):
        tag, i = _varint(b, i)
        wt, f = tag & 7, tag >> 3
        if wt == 4:
            raise ProtoError("end group for non-group")
        if f <= 0 or f > 0x1FFFFFFF:
            raise ProtoError("illegal tag")
        if wt == 0:
            v, i = _varint(b, i)
            yield f, wt, v
        elif wt == 1:
            if len(b) - i < 8:
                raise ProtoError("EOF")
            yield f, wt, struct.unpack_from("<Q", b, i)[0]
            i += 8
        elif wt == 2:
            n, i = _varint(b, i)
            if n > len(b) - i:
                raise ProtoError("EOF")
            yield f, wt, bytes(b[i:i + n])
            i += n
        elif wt == 5:
            if len(b) - i < 4:
                raise ProtoError("EOF")
            yield f, wt, struct.unpack_from("<I", b, i)[0]
            i += 4
        else:
            j = _skip(b, i, wt)
            yield f, wt, None
            i = j


def _expect(wt, want):
    if wt != want:
        raise ProtoError("wrong wireType")


def parse_anyvalue(b, cur=None, depth=0):
    """-> (kind, value): kind in string/bool/int/double/other/None; last oneof member wins."""
    kind, val = cur if cur else (None, None)
    for f, wt, v in fields(b):
        if f == 1:
            _expect(wt, 2)
            kind, val = "string", v
        elif f == 2:
            _expect(wt, 0)
            kind, val = "bool", v != 0
        elif f == 3:
            _expect(wt, 0)
            kind, val = "int", v - (1 << 64) if v >= 1 << 63 else v
        elif f == 4:
            _expect(wt, 1)
            kind, val = "double", struct.unpack("<d", struct.pack("<Q", v))[0]
        elif f == 5:
            _expect(wt, 2)
            for g, w2, x in fields(v):  # ArrayValue.values
                if g == 1:
                    _expect(w2, 2)
                    parse_anyvalue(x, None, depth + 1)
            kind, val = "other", None
        elif f == 6:
            _expect(wt, 2)
            for g, w2, x in fields(v):  # KeyValueList.values
                if g == 1:
                    _expect(w2, 2)
                    parse_kv(x, depth + 1)
            kind, val = "other", None
    return kind, val


def parse_kv(b, depth=0):
    key, val, has = b"", (None, None), False
    for f, wt, v in fields(b):
        if f == 1:
            _expect(wt, 2)
            key = v
        elif f == 2:
            _expect(wt, 2)
            val = parse_anyvalue(v, val if has else None, depth + 1)  # embedded message: merge
            has = True
    return key, (val if has else None)


def _validate(b, spec):
    for f, wt, v in fields(b):
        if f in spec:
            kind = spec[f]
            _expect(wt, {"varint": 0, "fixed64": 1}.get(kind, 2))
            if kind == "kv":
                parse_kv(v)


def parse_span(b):
    s = {"name": b"", "parent": b"", "start": 0, "end": 0, "code": 0, "attrs": []}
    for f, wt, v in fields(b):
        if f in (1, 2, 3):
            _expect(wt, 2)
        elif f == 4:
            _expect(wt, 2)
            s["parent"] = v
        elif f == 5:
            _expect(wt, 2)
            s["name"] = v
        elif f in (6, 10, 12, 14):
            _expect(wt, 0)
        elif f == 7:
            _expect(wt, 1)
            s["start"] = v
        elif f == 8:
            _expect(wt, 1)
            s["end"] = v
        elif f == 9:
            _expect(wt, 2)
            s["attrs"].append(parse_kv(v))
        elif f == 11:
            _expect(wt, 2)
            _validate(v, {1: "fixed64", 2: "bytes", 3: "kv", 4: "varint"})
        elif f == 13:
            _expect(wt, 2)
            _validate(v, {1: "bytes", 2: "bytes", 3: "bytes", 4: "kv", 5: "varint"})
        elif f == 15:
            _expect(wt, 2)
            for g, w2, x in fields(v):
                if g == 1:
                    _expect(w2, 0)
                elif g == 2:
                    _expect(w2, 2)
                elif g == 3:
                    _expect(w2, 0)
                    c = x & 0xFFFFFFFF
                    s["code"] = c - (1 << 32) if c >= 1 << 31 else c
    return s


def parse_batch(b):
    bt = {"resource": None, "spans": []}
    for f, wt, v in fields(b):
        if f == 1:
            _expect(wt, 2)
            if bt["resource"] is None:
                bt["resource"] = []
            for g, w2, x in fields(v):
                if g == 1:
                    _expect(w2, 2)
                    bt["resource"].append(parse_kv(x))
                elif g == 2:
                    _expect(w2, 0)
        elif f == 2:
            _expect(wt, 2)
            for g, w2, x in fields(v):  # InstrumentationLibrarySpans
                if g == 1:
                    _expect(w2, 2)
                    _validate(x, {1: "bytes", 2: "bytes"})
                elif g == 2:
                    _expect(w2, 2)
                    bt["spans"].append(parse_span(x))
    return bt


def prepare_for_read(body):
    """TraceBytes -> batches (PrepareForRead of both decoders after the header)."""
    batches = []
    for f, wt, v in fields(body):
        if f == 1:
            _expect(wt, 2)
            for g, w2, x in fields(v):  # tempopb.Trace
                if g == 1:
                    _expect(w2, 2)
                    batches.append(parse_batch(x))
    return batches


# ---- Go strconv ------------------------------------------------------------------------
_INT = re.compile(r"[+-]?[0-9]+\Z")
_DEC = re.compile(r"[+-]?(?:[0-9_]+\.?[0-9_]*|\.[0-9_]+)(?:[eE][+-]?[0-9_]+)?\Z")
_HEX = re.compile(r"[+-]?0[xX](?:[0-9a-fA-F_]+\.?[0-9a-fA-F_]*|\.[0-9a-fA-F_]+)[pP][+-]?[0-9_]+\Z")


def _underscore_ok(s):
    saw, i = "^", 0
    if s[:1] in ("+", "-"):
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i, saw, hexa = 2, "0", s[1].lower() == "x"
    while i < len(s):
        c = s[i]
        if c.isdigit() or (hexa and c.lower() in "abcdef"):
            saw = "0"
        elif c == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def parse_int(s):
    if not _INT.match(s):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def parse_float(s):
    body = s[1:] if s[:1] in "+-" else s
    if body.lower() in ("inf", "infinity"):
        return -math.inf if s[:1] == "-" else math.inf
    if s.lower() == "nan":
        return math.nan
    if _HEX.match(s):
        if "_" in s and not _underscore_ok(s):
            return None
        t = s.replace("_", "")
        neg = t[:1] == "-"
        t = t.lstrip("+-")
        if not re.search(r"[0-9a-fA-F]", t.split("p")[0].split("P")[0][2:]):
            return None
        v = float.fromhex(t)
        v = -v if neg else v
    elif _DEC.match(s):
        mant = re.split(r"[eE]", s)[0]
        if not re.search(r"[0-9]", mant):
            return None
        if "_" in s and not _underscore_ok(s):
            return None
        try:
            v = float(s.replace("_", ""))
        except ValueError:
            return None
    else:
        return None
    return None if math.isinf(v) else v


def parse_bool(s):
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return None


# ---- MatchesProto -----------------------------------------------------------------------
STATUS_CODE_MAPPING = {"unset": 0, "ok": 1, "error": 2}


def _match_attributes(tags, attrs):
    for key, val in attrs:
        k = key.decode("latin-1")
        if k not in tags:
            continue
        if val is None:  # (nil AnyValue: the reference dereferences it)
            continue
        search = tags[k]
        kind, v = val
        match = False
        if kind == "string":
            match = search.encode("latin-1") in v
        elif kind == "int":
            n = parse_int(search)
            match = n is not None and v == n
        elif kind == "double":
            f = parse_float(search)
            match = f is not None and v == f
        elif kind == "bool":
            bv = parse_bool(search)
            match = bv is not None and v == bv
        if match:
            del tags[k]


def _match_span(tags, s):
    if "name" in tags and tags["name"].encode("latin-1") == s["name"]:
        del tags["name"]
    if "error" in tags and tags["error"] == "true" and s["code"] == 2:
        del tags["error"]
    if "status.code" in tags and STATUS_CODE_MAPPING.get(tags["status.code"], 0) == s["code"]:
        del tags["status.code"]


def matches_proto(tid, batches, req):
    """trace.MatchesProto -> None or dict(trace_id, root_service_name, root_trace_name,
    start_time_unix_nano, duration_ms). Tags are handled as latin-1 strings (bytes)."""
    tstart, tend = (1 << 64) - 1, 0
    # (tags as byte strings: the engine receives them UTF-8 encoded)
    tags = {k.encode().decode("latin-1") if isinstance(k, str) else k.decode("latin-1"):
            v.encode().decode("latin-1") if isinstance(v, str) else v.decode("latin-1")
            for k, v in req.get("tags", {}).items()}
    root = root_batch = None
    for b in batches:
        if tags and b["resource"] is not None:
            _match_attributes(tags, b["resource"])
        for s in b["spans"]:
            tstart = min(tstart, s["start"])
            tend = max(tend, s["end"])
            if root is None and len(s["parent"]) == 0:
                root, root_batch = s, b
            if not tags:
                continue
            _match_span(tags, s)
            _match_attributes(tags, s["attrs"])
    if tags:
        return None
    sms, ems = tstart // 1000000, tend // 1000000
    dur = (ems - sms) & 0xFFFFFFFF  # uint32(traceEndMs - traceStartMs), uint64 wrap first
    mx, mn = req.get("max_ms", 0), req.get("min_ms", 0)
    if mx and mx < dur:
        return None
    if mn and mn > dur:
        return None
    if not (req.get("start", 0) <= ((ems // 1000) & 0xFFFFFFFF) and req.get("end", 0) >= ((sms // 1000) & 0xFFFFFFFF)):
        return None
    svc = name = ROOT_NOT_YET.encode()
    if root is not None:
        name = root["name"]
        for key, val in (root_batch["resource"] or []):
            if key == b"service.name":
                svc = val[1] if val is not None and val[0] == "string" else b""
                break
    return {"trace_id": tid, "root_service_name": svc, "root_trace_name": name,
            "start_time_unix_nano": tstart, "duration_ms": dur}


def decoder_matches(v2, tid, obj, req):
    """ObjectDecoder.Matches for dataEncoding v1 / v2; raises ProtoError where it errors."""
    if v2:
        if len(obj) < 8:
            raise ProtoError("buffer too short to have start/end")
        start, end = struct.unpack_from("<II", obj, 0)
        if not (req.get("start", 0) <= end and req.get("end", 0) >= start):
            return None
        d = (end - start) & 0xFFFFFFFF
        mx, mn = req.get("max_ms", 0), req.get("min_ms", 0)
        if mx and d > mx // 1000 + 1:
            return None
        if mn and d < mn // 1000:
            return None
        body = obj[8:]
    else:
        body = obj
    return matches_proto(tid, prepare_for_read(body), req)


# ---- the block -------------------------------------------------------------------------
def _snappy_framed(b):
    from oracle import oracle as O
    return O.snappy_framed_decode(b)


def _decompress(enc, payload):
    if enc == "none":
        return payload
    if enc == "snappy":
        return _snappy_framed(payload)
    if enc == "zstd":
        import pyarrow as pa
        return pa.input_stream(pa.py_buffer(payload), compression="zstd").read()
    raise ProtoError("unsupported encoding " + enc)


class ProtoBlock:
    def __init__(self, path):
        self.path = path
        meta = json.load(open(os.path.join(path, "meta.json")))
        self.enc = meta.get("encoding", "none")
        self.v2 = meta.get("dataEncoding") == "v2"
        if meta.get("dataEncoding") not in ("v1", "v2"):
            raise ProtoError("unknown dataEncoding")
        self.page_size = int(meta.get("indexPageSize", 0))
        self.total = int(meta.get("totalRecords", 0))
        self.index = open(os.path.join(path, "index"), "rb").read()
        self.data = open(os.path.join(path, "data"), "rb").read()

    def at(self, i):
        """indexReader.At -> (start, length) | None; raises ProtoError on a bad page/record."""
        import xxhash
        if i < 0 or i >= self.total:
            return None
        per = (self.page_size - 8 - 6) // 28 if self.page_size > 14 else 0
        if per == 0:
            raise ProtoError("index page size")
        p, r = divmod(i, per)
        off = p * self.page_size
        if off + self.page_size > len(self.index):
            raise ProtoError("index short read")
        pg = self.index[off:off + self.page_size]
        total, hl = struct.unpack_from("<IH", pg, 0)
        if hl != 8 or total - 14 != len(pg) - 14:
            raise ProtoError("index page framing")
        data = pg[14:]
        if struct.unpack_from("<Q", pg, 6)[0] != xxhash.xxh64(data).intdigest():
            raise ProtoError("mismatched checksum")
        if (r + 1) * 28 > len(data):
            raise ProtoError("record out of bounds")
        rec = data[r * 28:(r + 1) * 28]
        if rec == bytes(28):
            raise ProtoError("zero record")
        return struct.unpack_from("<QI", rec, 16)

    def page(self, start, length):
        """dataReader.Read of one record: page framing, then decompression."""
        if start + length > len(self.data):
            raise ProtoError("record out of bounds")
        b = self.data[start:start + length]
        if len(b) < 6:
            raise ProtoError("page too short")
        total, hl = struct.unpack_from("<IH", b, 0)
        if hl != 0 or total != len(b):
            raise ProtoError("page framing")
        try:
            return _decompress(self.enc, b[6:])
        except ProtoError:
            raise
        except Exception as e:  # noqa: BLE001  (codec errors)
            raise ProtoError("decompress: %s" % e)

    def search(self, tags=None, min_ms=0, max_ms=0, start=0, end=0, limit=20, start_page=0, total_pages=0,
               max_bytes=0, chunk_size_bytes=1_000_000):
        """BackendBlock.Search -> (traces, metrics) or raises ProtoError. traces: dicts with
        trace_id (bytes), root_service_name/root_trace_name (bytes), start_time_unix_nano,
        duration_ms, object_idx."""
        req = {"tags": {k: v for k, v in (tags or {}).items()}, "min_ms": min_ms, "max_ms": max_ms,
               "start": start, "end": end}
        cur = start_page if total_pages > 0 else 0
        maxp = cur + total_pages if total_pages > 0 else 1 << 62
        out, met = [], {"inspected_traces": 0, "inspected_bytes": 0, "skipped_traces": 0}
        obj_idx = sum(self._objects_before(cur))
        while True:
            if cur >= maxp:
                return out, met
            rec = self.at(cur)
            if rec is None:
                return out, met
            records, length = [], 0
            while rec is not None:
                if (length + rec[1] > chunk_size_bytes or cur >= maxp) and records:
                    break
                records.append(rec)
                length += rec[1]
                cur += 1
                rec = self.at(cur)
            pages = [self.page(s, l) for s, l in records]
            for pg in pages:
                i = 0
                while i < len(pg):
                    if len(pg) - i < 8:
                        raise ProtoError("object framing")
                    tl, il = struct.unpack_from("<II", pg, i)
                    rest = (tl - 8) & 0xFFFFFFFF
                    if len(pg) - i - 8 < rest or il > rest:
                        raise ProtoError("object framing")
                    tid = pg[i + 8:i + 8 + il]
                    obj = pg[i + 8 + il:i + 8 + rest]
                    i += 8 + rest
                    met["inspected_traces"] += 1
                    met["inspected_bytes"] += len(obj)
                    if max_bytes > 0 and len(obj) > max_bytes:
                        met["skipped_traces"] += 1
                    else:
                        m = decoder_matches(self.v2, tid, obj, req)
                        if m is not None:
                            m["object_idx"] = obj_idx
                            out.append(m)
                    obj_idx += 1
                    if len(out) >= limit:
                        return out, met

    def _objects_before(self, page):
        """object counts of the pages before `page` (for object_idx; pages read whole)."""
        for p in range(page):
            rec = self.at(p)
            pg = self.page(*rec)
            n, i = 0, 0
            while i + 8 <= len(pg):
                tl = struct.unpack_from("<I", pg, i)[0]
                i += tl
                n += 1
            yield n


# ---- test-data writer: tempopb protos (test tooling) -----------------------------------
def _vint(v):
    v &= 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while True:
        c = v & 0x7F
        v >>= 7
        if v:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _fld(f, wt):
    return _vint((f << 3) | wt)


def _ld(f, b):
    return _fld(f, 2) + _vint(len(b)) + b


def enc_anyvalue(v):
    if isinstance(v, bool):
        return _fld(2, 0) + _vint(int(v))
    if isinstance(v, int):
        return _fld(3, 0) + _vint(v)
    if isinstance(v, float):
        return _fld(4, 1) + struct.pack("<d", v)
    if isinstance(v, (str, bytes)):
        return _ld(1, v.encode() if isinstance(v, str) else v)
    if isinstance(v, list):
        return _ld(5, b"".join(_ld(1, enc_anyvalue(x)) for x in v))
    raise TypeError(v)


def enc_kv(k, v):
    return _ld(1, k.encode() if isinstance(k, str) else k) + (b"" if v is None else _ld(2, enc_anyvalue(v)))


def enc_span(s):
    b = _ld(1, s.get("trace_id", b"\x01" * 16)) + _ld(2, s.get("span_id", b"\x02" * 8))
    if s.get("parent"):
        b += _ld(4, s["parent"])
    b += _ld(5, s.get("name", "").encode() if isinstance(s.get("name", ""), str) else s["name"])
    b += _fld(6, 0) + _vint(s.get("kind", 1))
    b += _fld(7, 1) + struct.pack("<Q", s.get("start", 0)) + _fld(8, 1) + struct.pack("<Q", s.get("end", 0))
    for k, v in s.get("attrs", {}).items():
        b += _ld(9, enc_kv(k, v))
    if "code" in s and s["code"] is not None:
        b += _ld(15, _ld(2, b"msg") + _fld(3, 0) + _vint(s["code"]))
    return b


def enc_batch(bt):
    b = b""
    if bt.get("resource") is not None:
        b += _ld(1, b"".join(_ld(1, enc_kv(k, v)) for k, v in bt["resource"].items()))
    ils = _ld(1, _ld(1, b"lib") + _ld(2, b"1.0")) + b"".join(_ld(2, enc_span(s)) for s in bt.get("spans", []))
    return b + _ld(2, ils)


def enc_trace(batches):
    return b"".join(_ld(1, enc_batch(bt)) for bt in batches)


def enc_object(batches, v2, start=0, end=0, split=1):
    """A stored object: TraceBytes of `split` marshalled Traces (batches dealt round-robin),
    with the v2 start/end header when v2."""
    parts = [[] for _ in range(max(1, split))]
    for i, bt in enumerate(batches):
        parts[i % len(parts)].append(bt)
    tb = b"".join(_ld(1, enc_trace(p)) for p in parts)
    return (struct.pack("<II", start, end) + tb) if v2 else tb
