"""The C ABI library: builds, loads, exports every symbol include/tsg.h declares,
refuses to run without a device, and its host logic (request normalisation,
block prefilter, writer) agrees with the oracle. CPU only: no compute call."""
import os
import re

import pytest

from oracle import oracle as O
import tempo_amd as T
from tempo_amd import tsg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "tsg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tsg_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    L = T.lib()
    syms = header_symbols()
    assert len(syms) >= 29
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(tsg.EXPORTED) == syms


def test_shim_pattern_driver_loads():
    """libtsg_shim_pattern.so (the shim's per-block call pattern for the bench) binds to
    the same libtsg: one copy of the library in the process."""
    S = tsg.shim_pattern_lib()
    assert hasattr(S, "tsgx_shim_pattern")
    maps = open("/proc/self/maps").read()
    assert len({ln.split()[-1] for ln in maps.splitlines() if ln.endswith("/libtsg.so")}) == 1


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    with pytest.raises(T.TsgError) as e:
        T.Engine()
    assert e.value.code == tsg.TSG_E_DEVICE


def test_abi_version():
    assert T.lib().tsg_abi_version() == 7


def test_struct_layouts_match_header(tmp_path):
    # the ctypes mirrors of the ABI-7 structs against the compiled header (gcc, no GPU)
    import ctypes as C
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tsg.h"\nint main(void){printf("%zu %zu %zu %zu %zu\\n",'
                   ' sizeof(tsg_metrics), sizeof(tsg_result), offsetof(tsg_result, nblocks), sizeof(tsg_search_item),'
                   ' offsetof(tsg_metrics, path));return 0;}\n')
    exe = tmp_path / "sz"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.check_call(["gcc", "-I", inc, str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [C.sizeof(tsg._Metrics), C.sizeof(tsg._Result), tsg._Result.nblocks.offset, C.sizeof(tsg._SearchItem),
                   tsg._Metrics.path.offset]


def test_debug_set_rejects_unknown_hooks():
    with pytest.raises(T.TsgError) as e:
        T.debug_set("no_such_hook", 1)
    assert e.value.code == tsg.TSG_E_INVALID
    T.debug_set("res_torn", 0)  # (a known hook: accepted without a device)


@pytest.mark.parametrize("req,terms", [
    ({"error": "true"}, [(b"status.code", b"2")]),
    ({"error": "false"}, [(b"error", b"false")]),
    ({"status.code": "error"}, [(b"status.code", b"2")]),
    ({"status.code": "ok"}, [(b"status.code", b"1")]),
    ({"status.code": "unset"}, [(b"status.code", b"0")]),
    ({"status.code": "bogus"}, [(b"status.code", b"bogus")]),
    ({"Service.Name": "SVC-07"}, [(b"service.name", b"svc-07")]),
    ({"Error": "true"}, [(b"error", b"true")]),  # rewrite matches the request key before ToLower
    ({"x-dbg-exhaustive": "!"}, []),
    ({"k": ""}, [(b"k", b"")]),
    ({"ÄÖ": "ÉŸ"}, [("äö".encode(), "éÿ".encode())]),
])
def test_pipeline_normalisation(req, terms):
    p = T.Pipeline(T.SearchRequest(tags=req))
    assert p.terms() == terms
    q = p.query.contents
    assert q.exhaustive == (1 if "x-dbg-exhaustive" in req else 0)


def test_pipeline_filters_flags():
    q = T.Pipeline(T.SearchRequest(min_duration_ms=10, max_duration_ms=0, start=5, end=0)).query.contents
    assert (q.has_min, q.has_max, q.has_range, q.min_ns) == (1, 0, 0, 10_000_000)
    q = T.Pipeline(T.SearchRequest(max_duration_ms=90_000, start=5, end=9)).query.contents
    assert (q.has_min, q.has_max, q.has_range, q.max_ns, q.start_s, q.end_s) == (0, 1, 1, 90_000_000_000, 5, 9)


def test_block_prefilter_matches_oracle(golden):
    blk = golden["pipeline"]["block"]
    h = blk["header"]
    hdr = T.fb_search_header([{"id": b"a", "start": 0, "end": h["min_dur_ns"], "tags": h["tags"]},
                              {"id": b"b", "start": 0, "end": h["max_dur_ns"], "tags": h["tags"]}])
    for c in blk["cases"]:
        req = T.SearchRequest(tags=c["req"], min_duration_ms=c["min"], max_duration_ms=c["max"])
        assert T.Pipeline(req).matches_block(hdr) == c["match"], c["name"]
        assert O.pipeline_matches_block(hdr, tags=c["req"], min_ms=c["min"], max_ms=c["max"]) == c["match"]


def test_header_min_dur_quirk():
    """SearchBlockHeaderMutable.AddEntry: after a zero-duration entry the next one
    overwrites MinDur (pkg/tempofb/SearchBlockHeader_util.go:37-43, pitfall P1)."""
    import struct
    hdr = T.fb_search_header([{"id": b"a", "start": 5, "end": 10}, {"id": b"b", "start": 7, "end": 7},
                              {"id": b"c", "start": 0, "end": 500}])
    # min = 5 -> 0 (dur 0 < 5) -> 500 (MinDur == 0 is treated as unset)
    req = T.SearchRequest(max_duration_ms=0)
    p = T.Pipeline(T.SearchRequest(tags={}, max_duration_ms=1))
    assert p.matches_block(hdr)  # MinDur = 500 ns <= 1 ms
    # the oracle reads the same stored value
    assert O.pipeline_matches_block(hdr, max_ms=1)


def test_writer_entry_is_readable_flatbuffer():
    fb = T.fb_search_entry({"id": b"\x01\x02", "start": 3, "end": 9, "tags": {"a": ["x", "y"], "b": ["z"]}})
    assert O.contains_tag_entry(fb, b"a", b"y")
    assert O.contains_tag_entry(fb, b"b", b"")
    assert not O.contains_tag_entry(fb, b"c", b"")
