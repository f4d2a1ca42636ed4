"""Proto-object search oracle pinned to the reference's known answers (CPU).

TestMatches (pkg/model/object_decoder_test.go:49-478): one two-batch trace, 32 requests,
both object encodings (v1 TraceBytes, v2 with the start/end header 10..20 s), expected
TraceSearchMetadata or nil. TestMatchesFails (:480-485): a 2-byte object is an error for
both. Plus the engine's host-side Go strconv against the oracle's restatement (the same
strings, both must agree on acceptance and value).
"""
import math
import struct

import pytest

from oracle import proto_oracle as P
import tempo_amd as T

SEC = 1_000_000_000
TEST_TRACE = [
    {"resource": {"service.name": "svc", "cluster": "prod"},
     "spans": [{"name": "test", "start": 10 * SEC, "end": 20 * SEC, "code": 1,
                "attrs": {"foo": "barricus", "intfoo": 42, "floatfoo": 42.42, "boolfoo": True}}]},
    {"resource": {"service.name": "svc2"},
     "spans": [{"name": "test2", "start": 10 * SEC, "end": 20 * SEC, "code": 1,
                "attrs": {"foo2": "barricus2"}}]},
]
META = {"trace_id": b"\x01", "root_service_name": b"svc", "root_trace_name": b"test",
        "start_time_unix_nano": 10 * SEC, "duration_ms": 10000}

# (name, request, matches) — the table of TestMatches
CASES = [
    ("range before doesn't match", dict(start=0, end=5), False),
    ("range after doesn't match", dict(start=25, end=30), False),
    ("encompassing range matches", dict(start=5, end=30), True),
    ("encompassed range matches", dict(start=12, end=15), True),
    ("overlap start matches", dict(start=8, end=15), True),
    ("overlap end matches", dict(start=12, end=25), True),
    ("max duration excludes", dict(start=12, end=15, max_ms=1), False),
    ("max duration includes", dict(start=12, end=15, max_ms=10000), True),
    ("min duration excludes", dict(start=12, end=15, max_ms=1, min_ms=10000), False),
    ("min duration includes", dict(start=12, end=15, max_ms=10000, min_ms=5000), True),
    ("string tag excludes", dict(start=12, end=15, tags={"foo": "baz"}), False),
    ("string tag includes", dict(start=12, end=15, tags={"foo": "bar"}), True),
    ("resource tag includes", dict(start=12, end=15, tags={"service.name": "svc"}), True),
    ("int tag excludes", dict(start=12, end=15, tags={"intfoo": "blerg"}), False),
    ("int tag includes", dict(start=12, end=15, tags={"intfoo": "42"}), True),
    ("float tag excludes", dict(start=12, end=15, tags={"floatfoo": "42.4323"}), False),
    ("float tag includes", dict(start=12, end=15, tags={"floatfoo": "42.42"}), True),
    ("bool tag excludes", dict(start=12, end=15, tags={"boolfoo": "False"}), False),
    ("bool tag includes", dict(start=12, end=15, tags={"boolfoo": "true"}), True),
    ("one includes/one excludes", dict(start=12, end=15, tags={"foo": "bar", "boolfoo": "False"}), False),
    ("one includes/resource tag excludes", dict(start=12, end=15, tags={"foo": "bar", "service.name": "blerg"}), False),
    ("both include. one resource tag", dict(start=12, end=15, tags={"foo": "bar", "service.name": "svc"}), True),
    ("both include", dict(start=12, end=15, tags={"foo": "bar", "boolfoo": "true"}), True),
    ("both include across batches", dict(start=12, end=15, tags={"foo": "bar", "service.name": "svc2"}), True),
    ("two resource tags. one excludes", dict(start=12, end=15, tags={"cluster": "prod", "service.name": "not"}), False),
    ("name includes", dict(start=12, end=15, tags={"name": "test"}), True),
    ("name excludes", dict(start=12, end=15, tags={"name": "no"}), False),
    ("name excludes with resource tag", dict(start=12, end=15, tags={"name": "no", "cluster": "prod"}), False),
    ("name excludes with span tag", dict(start=12, end=15, tags={"name": "no", "foo": "barricus"}), False),
    ("error excludes", dict(start=12, end=15, tags={"error": "true"}), False),
    ("status.code excludes", dict(start=12, end=15, tags={"status.code": "error"}), False),
    ("status.code includes", dict(start=12, end=15, tags={"status.code": "ok"}), True),
]


@pytest.mark.parametrize("v2", [False, True], ids=["v1", "v2"])
@pytest.mark.parametrize("name,req,ok", CASES, ids=[c[0] for c in CASES])
def test_matches_table(name, req, ok, v2):
    obj = P.enc_object(TEST_TRACE, v2, 10, 20)
    got = P.decoder_matches(v2, b"\x01", obj, req)
    assert (got == META) if ok else got is None
    if ok:
        assert got["trace_id"].hex().lstrip("0") == "1"  # TraceID "1"


@pytest.mark.parametrize("v2", [False, True])
def test_matches_fails(v2):
    with pytest.raises(P.ProtoError):
        P.decoder_matches(v2, b"\x01", b"\x02\x03", {})


def test_root_and_time_semantics():
    # no root span: both names are the placeholder; traceStart/End over every span
    tr = [{"resource": {"service.name": "a"},
           "spans": [{"name": "x", "parent": b"\x09", "start": 5 * SEC, "end": 7 * SEC},
                     {"name": "y", "parent": b"\x09", "start": 3 * SEC, "end": 6 * SEC}]}]
    m = P.decoder_matches(False, b"\x00\x02", P.enc_object(tr, False), dict(start=0, end=100))
    assert m["root_service_name"] == m["root_trace_name"] == P.ROOT_NOT_YET.encode()
    assert m["start_time_unix_nano"] == 3 * SEC and m["duration_ms"] == 4000
    # the first span with an empty parent wins; its batch's service.name (non-string -> "")
    tr2 = [{"resource": {"service.name": 7}, "spans": [{"name": "r", "start": SEC, "end": 2 * SEC}]},
           {"resource": {"service.name": "b"}, "spans": [{"name": "r2", "start": SEC, "end": 2 * SEC}]}]
    m = P.decoder_matches(False, b"\x03", P.enc_object(tr2, False), dict(start=0, end=100))
    assert m["root_service_name"] == b"" and m["root_trace_name"] == b"r"
    # status.code with an unknown value maps to UNSET (StatusCodeMapping zero value)
    tr3 = [{"resource": {}, "spans": [{"name": "s", "start": SEC, "end": 2 * SEC, "code": 0}]}]
    assert P.decoder_matches(False, b"\x04", P.enc_object(tr3, False),
                             dict(start=0, end=100, tags={"status.code": "bogus"})) is not None
    # TraceBytes holding several Traces: batches concatenate (PrepareForRead)
    obj = P.enc_object(TEST_TRACE, True, 10, 20, split=2)
    assert P.decoder_matches(True, b"\x01", obj, dict(start=12, end=15, tags={"foo": "bar", "service.name": "svc2"})) == META


GO_STRINGS = ["0", "42", "-42", "+7", "", "-", "4 2", " 42", "9223372036854775807", "9223372036854775808",
              "-9223372036854775808", "-9223372036854775809", "1_000", "0x10", "42.42", "42.4323", ".5", "5.", ".",
              "1e10", "1E-3", "1e", "1e+", "inf", "+Inf", "-infinity", "INFINITY", "infi", "nan", "NaN", "-nan",
              "0x1p-2", "0X1.8P1", "0x1.8", "0x", "0xp1", "1_0.5", "_1", "1_", "1__0", "1e1_0", "1e400", "-1e400",
              "4.9e-324", "1e-400", "true", "True", "TRUE", "t", "T", "1", "false", "f", "F", "0", "tRUE", "yes",
              "0.1", "123456789012345678901234567890", "0x_1p0", "0x1_0p0", "+0x1p1"]


@pytest.mark.parametrize("s", GO_STRINGS)
def test_go_strconv_engine_vs_oracle(s):
    ok, v = T.go_parse("int", s)
    e = P.parse_int(s)
    assert ok == (e is not None) and (not ok or v == e)
    ok, v = T.go_parse("float", s)
    e = P.parse_float(s)
    assert ok == (e is not None), s
    if ok:
        assert (math.isnan(v) and math.isnan(e)) or (v == e and math.copysign(1, v) == math.copysign(1, e))
    ok, v = T.go_parse("bool", s)
    e = P.parse_bool(s)
    assert ok == (e is not None) and (not ok or v == e)


def test_go_strconv_known_values():
    assert P.parse_int("9223372036854775807") == 2 ** 63 - 1 and P.parse_int("9223372036854775808") is None
    assert P.parse_float("0x1p-2") == 0.25 and P.parse_float("1e400") is None and P.parse_float("-Inf") == -math.inf
    assert P.parse_float("0x1.8") is None  # hex mantissa needs a p exponent
    assert P.parse_bool("True") is True and P.parse_bool("tRUE") is None
    assert P.parse_float("4.9e-324") == struct.unpack("<d", struct.pack("<Q", 1))[0]
