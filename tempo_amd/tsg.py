"""ctypes binding of libtsg (include/tsg.h) — the host mirror of Tempo's search
operator interface for this path.

Names follow the reference: ``SearchRequest`` (tempopb.SearchRequest,
pkg/tempopb/tempo.proto:44-52), ``Pipeline`` (search.NewSearchPipeline,
tempodb/search/pipeline.go:26), ``BackendSearchBlock`` with ``search``/``tags``/
``tag_values`` (tempodb/search/backend_search_block.go:132-298, the
SearchableBlock interface of searchable_block.go:7-11), ``Results`` metrics
(tempodb/search/results.go:110-140) and ``TraceSearchMetadata``.

There is no CPU search path: importing works anywhere (the writer/synthetic
tooling is host code), but ``Engine()`` raises if no HIP device is visible or
the native library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import weakref
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSG_LIB_PATH") or os.path.join(HERE, "libtsg.so")  # (override: A/B runs of two builds)

TSG_OK = 0
TSG_E_NOT_FOUND = 1
TSG_E_CORRUPT = 2
TSG_E_UNSUPPORTED_ENCODING = 3
TSG_E_DEVICE = 4
TSG_E_CANCELLED = 5
TSG_E_OOM = 6
TSG_E_INVALID = 7
TSG_E_UNSUPPORTED = 8
TSG_E_IO = 9

ENC_NONE = 0
ENC_SNAPPY = 6
ENC_NAMES = ["none", "gzip", "lz4-64k", "lz4-256k", "lz4-1M", "lz4", "snappy", "zstd", "s2"]  # backend.Encoding.String

SEARCH_TIME_SCAN = 1  # tsg_search_opts.flags: HIP events around the scan kernel
SEARCH_TIME_ALL = 2   # ... and around the whole device sequence
SEARCH_TIME_DEFER = 4  # events around the search kernel, read later by Engine.kernel_times()

PATH_RESIDENT = 1  # tsg_metrics.path (ABI 7): search_resident_kernel served (part of) the search
PATH_PLAIN = 2     # search_pool_kernel / search_static_kernel as plain launches
PATH_OTHER = 4     # search_fast_kernel, the dictionary pass, the general path
PATH_COTENANT = 8  # the resident kernel declined: another process has a context on the GPU


class TsgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"tsg error {code}: {msg}")
        self.code = code


class _Options(C.Structure):
    _fields_ = [("num_devices", C.c_int32), ("devices", C.POINTER(C.c_int32)), ("flags", C.c_uint32)]


class _Request(C.Structure):
    _fields_ = [("ntags", C.c_uint32),
                ("tag_keys", C.POINTER(C.c_char_p)), ("tag_key_lens", C.POINTER(C.c_uint32)),
                ("tag_values", C.POINTER(C.c_char_p)), ("tag_value_lens", C.POINTER(C.c_uint32)),
                ("min_duration_ms", C.c_uint32), ("max_duration_ms", C.c_uint32),
                ("limit", C.c_uint32), ("start", C.c_uint32), ("end", C.c_uint32)]


class _Query(C.Structure):
    _fields_ = [("nterms", C.c_uint32),
                ("keys", C.POINTER(C.POINTER(C.c_uint8))), ("key_lens", C.POINTER(C.c_uint32)),
                ("values", C.POINTER(C.POINTER(C.c_uint8))), ("value_lens", C.POINTER(C.c_uint32)),
                ("has_min", C.c_uint8), ("has_max", C.c_uint8), ("has_range", C.c_uint8),
                ("exhaustive", C.c_uint8), ("min_ns", C.c_uint64), ("max_ns", C.c_uint64),
                ("start_s", C.c_uint32), ("end_s", C.c_uint32)]


class _Metrics(C.Structure):
    _fields_ = [("traces_inspected", C.c_uint32), ("blocks_inspected", C.c_uint32),
                ("blocks_skipped", C.c_uint32), ("reruns", C.c_uint32), ("bytes_inspected", C.c_uint64),
                ("device_bytes_read", C.c_uint64), ("kernel_ns", C.c_uint64),
                ("scan_kernel_ns", C.c_uint64), ("scan_bytes", C.c_uint64),
                ("path", C.c_uint32), ("reserved", C.c_uint32)]


class _Result(C.Structure):
    _fields_ = [("n", C.c_uint64), ("trace_id", C.POINTER(C.c_uint8)), ("trace_id_len", C.POINTER(C.c_uint8)),
                ("start_ns", C.POINTER(C.c_uint64)), ("end_ns", C.POINTER(C.c_uint64)),
                ("duration_ms", C.POINTER(C.c_uint32)), ("block_idx", C.POINTER(C.c_uint32)),
                ("entry_idx", C.POINTER(C.c_uint64)),
                ("root_service", C.POINTER(C.c_char_p)), ("root_service_len", C.POINTER(C.c_uint32)),
                ("root_name", C.POINTER(C.c_char_p)), ("root_name_len", C.POINTER(C.c_uint32)),
                ("metrics", _Metrics), ("nblocks", C.c_uint64), ("block_status", C.POINTER(C.c_int32)),
                ("block_error", C.POINTER(C.c_char_p)), ("names", C.c_void_p), ("names_len", C.c_uint64),
                ("root_service_off", C.POINTER(C.c_uint64)), ("root_name_off", C.POINTER(C.c_uint64))]


class _SearchOpts(C.Structure):
    _fields_ = [("limit", C.c_uint32), ("flags", C.c_uint32), ("query_id", C.c_uint64),
                ("seen_ids", C.c_void_p), ("nseen", C.c_uint64)]


class _SearchItem(C.Structure):
    _fields_ = [("blocks", C.c_void_p), ("nblocks", C.c_size_t), ("query", C.c_void_p), ("opts", _SearchOpts)]


class _BlockInfo(C.Structure):
    _fields_ = [("entries", C.c_uint64), ("pages", C.c_uint64), ("keys", C.c_uint64),
                ("header_bytes", C.c_uint64), ("fb_bytes", C.c_uint64), ("device_bytes", C.c_uint64),
                ("min_dur_ns", C.c_uint64), ("max_dur_ns", C.c_uint64), ("device", C.c_int32),
                ("encoding", C.c_int32), ("streaming", C.c_int32), ("partial", C.c_int32),
                ("stop_status", C.c_int32), ("index_truncated", C.c_int32), ("live", C.c_int32),
                ("hdr_deferred", C.c_int32), ("traces", C.c_uint64)]


class _LookupOpts(C.Structure):
    _fields_ = [("time_start", C.c_uint32), ("time_end", C.c_uint32),
                ("block_start", C.c_char_p), ("block_end", C.c_char_p)]


class _FindResult(C.Structure):
    _fields_ = [("n", C.c_uint64), ("id_idx", C.POINTER(C.c_uint32)), ("block_idx", C.POINTER(C.c_uint32)),
                ("status", C.POINTER(C.c_int32)), ("obj_off", C.POINTER(C.c_uint64)),
                ("obj_len", C.POINTER(C.c_uint32)), ("obj_bytes", C.POINTER(C.c_uint8)), ("kernel_ns", C.c_uint64)]


class _ProtoRequest(C.Structure):
    _fields_ = [("ntags", C.c_uint32), ("keys", C.POINTER(C.c_char_p)), ("key_lens", C.POINTER(C.c_uint32)),
                ("values", C.POINTER(C.c_char_p)), ("value_lens", C.POINTER(C.c_uint32)),
                ("min_duration_ms", C.c_uint32), ("max_duration_ms", C.c_uint32), ("start", C.c_uint32),
                ("end", C.c_uint32), ("limit", C.c_uint32), ("start_page", C.c_uint32), ("total_pages", C.c_uint32),
                ("max_bytes", C.c_uint32), ("chunk_size_bytes", C.c_uint32)]


class _ProtoResult(C.Structure):
    _fields_ = [("n", C.c_uint32), ("trace_ids", C.POINTER(C.c_uint8)), ("trace_id_off", C.POINTER(C.c_uint32)),
                ("trace_id_len", C.POINTER(C.c_uint32)), ("root_service_name", C.POINTER(C.c_void_p)),
                ("root_trace_name", C.POINTER(C.c_void_p)), ("start_time_unix_nano", C.POINTER(C.c_uint64)),
                ("duration_ms", C.POINTER(C.c_uint32)), ("object_idx", C.POINTER(C.c_uint32)),
                ("inspected_traces", C.c_uint64), ("inspected_bytes", C.c_uint64), ("skipped_traces", C.c_uint64),
                ("kernel_ns", C.c_uint64), ("root_service_name_len", C.POINTER(C.c_uint32)),
                ("root_trace_name_len", C.POINTER(C.c_uint32))]


class _LookupResult(C.Structure):
    _fields_ = [("n", C.c_uint64), ("id_idx", C.POINTER(C.c_uint32)), ("block_idx", C.POINTER(C.c_uint32)),
                ("record_idx", C.POINTER(C.c_int32)), ("record_start", C.POINTER(C.c_uint64)),
                ("record_length", C.POINTER(C.c_uint32)), ("kernel_ns", C.c_uint64)]


# Every symbol include/tsg.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "tsg_init", "tsg_shutdown", "tsg_device_count", "tsg_device_numa_node", "tsg_device_counters", "tsg_last_error", "tsg_abi_version", "tsg_cancel",
    "tsg_pipeline_new", "tsg_pipeline_query", "tsg_pipeline_free", "tsg_pipeline_matches_header",
    "tsg_block_open", "tsg_block_open_pages", "tsg_block_open_mem", "tsg_block_clone", "tsg_wal_block_open", "tsg_wal_block_open_mem", "tsg_block_close", "tsg_block_info_get", "tsg_block_tags",
    "tsg_block_tag_values", "tsg_free", "tsg_search", "tsg_result_free", "tsg_kernel_times", "tsg_results_combine",
    "tsg_v2block_open", "tsg_v2block_close", "tsg_lookup_ids", "tsg_lookup_result_free", "tsg_find_ids",
    "tsg_find_result_free", "tsg_proto_block_open", "tsg_proto_block_close", "tsg_proto_block_info",
    "tsg_proto_search", "tsg_proto_result_free", "tsg_go_parse", "tsg_write_v2_block",
    "tsg_write_search_block", "tsg_write_wal_search", "tsg_fb_search_entry", "tsg_fb_search_header", "tsg_synth_search_block",
    "tsg_synth_v2_block", "tsg_live_block_open_mem", "tsg_search_tags", "tsg_search_tag_values",
    "tsg_result_pack", "tsg_wire_merge", "tsg_search_batch", "tsg_debug_set",
    "tsg_shm_open", "tsg_shm_close", "tsg_shm_put", "tsg_shm_merge",
]

_lib = None


def lib():
    """Load libtsg.so; raises (loudly) if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libtsg.so not built at {LIB_PATH}: run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        vp, u8p = C.c_void_p, C.POINTER(C.c_uint8)
        L.tsg_last_error.restype = C.c_char_p
        L.tsg_init.argtypes = [C.POINTER(_Options), C.POINTER(vp)]
        L.tsg_shutdown.argtypes = [vp]
        L.tsg_device_count.argtypes = [vp]
        L.tsg_device_numa_node.argtypes = [vp, C.c_int]
        L.tsg_cancel.argtypes = [vp, C.c_uint64]
        L.tsg_pipeline_new.argtypes = [C.POINTER(_Request), C.POINTER(vp)]
        L.tsg_pipeline_query.argtypes = [vp]
        L.tsg_pipeline_query.restype = C.POINTER(_Query)
        L.tsg_pipeline_free.argtypes = [vp]
        L.tsg_pipeline_matches_header.argtypes = [C.POINTER(_Query), C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        L.tsg_block_open.argtypes = [vp, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.tsg_device_counters.argtypes = [vp, C.c_int, C.POINTER(C.c_uint64), C.c_size_t]
        L.tsg_block_open_pages.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(vp)]
        L.tsg_block_close.argtypes = [vp]
        L.tsg_block_clone.argtypes = [vp, vp, C.c_int, C.POINTER(vp)]
        L.tsg_wal_block_open.argtypes = [vp, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.tsg_wal_block_open_mem.argtypes = [vp, C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(vp)]
        L.tsg_write_wal_search.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int]
        L.tsg_block_info_get.argtypes = [vp, C.POINTER(_BlockInfo)]
        L.tsg_live_block_open_mem.argtypes = [vp, C.c_char_p, vp, C.c_size_t, vp, C.c_size_t, C.c_int, C.POINTER(vp)]
        L.tsg_result_pack.argtypes = [C.POINTER(_Result), C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.tsg_wire_merge.argtypes = [C.POINTER(u8p), C.POINTER(C.c_size_t), C.c_size_t, C.c_uint64, C.c_uint64,
                                     vp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.tsg_search_tags.argtypes = [C.POINTER(vp), C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_size_t)]
        L.tsg_search_tag_values.argtypes = [C.POINTER(vp), C.c_size_t, C.c_char_p, C.c_size_t, C.c_int64,
                                            C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.tsg_block_tags.argtypes = [vp, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.tsg_block_tag_values.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                           C.POINTER(C.c_size_t)]
        L.tsg_free.argtypes = [vp]
        L.tsg_search.argtypes = [vp, C.POINTER(vp), C.c_size_t, C.POINTER(_Query), C.POINTER(_SearchOpts),
                                 C.POINTER(C.POINTER(_Result))]
        L.tsg_result_free.argtypes = [C.POINTER(_Result)]
        L.tsg_search_batch.argtypes = [vp, C.POINTER(_SearchItem), C.c_size_t, C.c_uint32,
                                       C.POINTER(C.POINTER(_Result)), C.POINTER(C.c_uint64)]
        L.tsg_debug_set.argtypes = [C.c_char_p, C.c_int64]
        L.tsg_shm_open.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.POINTER(vp)]
        L.tsg_shm_close.argtypes = [vp]
        L.tsg_shm_put.argtypes = [vp, C.c_uint32, vp, C.c_size_t, C.c_double]
        L.tsg_shm_merge.argtypes = [vp, C.c_uint32, C.c_uint64, C.c_uint64, vp, C.c_size_t, C.POINTER(C.c_size_t),
                                    C.c_double]
        L.tsg_kernel_times.argtypes = [vp, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_size_t)]
        L.tsg_results_combine.argtypes = [C.POINTER(_Result), C.c_uint32, C.POINTER(C.POINTER(_Result))]
        L.tsg_v2block_open.argtypes = [vp, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.tsg_v2block_close.argtypes = [vp]
        L.tsg_lookup_ids.argtypes = [vp, C.POINTER(vp), C.c_size_t, vp, C.c_size_t, C.POINTER(_LookupOpts),
                                     C.POINTER(C.POINTER(_LookupResult))]
        L.tsg_lookup_result_free.argtypes = [C.POINTER(_LookupResult)]
        L.tsg_find_ids.argtypes = [vp, C.POINTER(vp), C.c_size_t, vp, C.c_size_t, C.POINTER(_LookupOpts),
                                   C.POINTER(C.POINTER(_FindResult))]
        L.tsg_find_result_free.argtypes = [C.POINTER(_FindResult)]
        L.tsg_proto_block_open.argtypes = [vp, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.tsg_proto_block_close.argtypes = [vp]
        L.tsg_proto_block_info.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.tsg_proto_search.argtypes = [vp, vp, C.POINTER(_ProtoRequest), C.POINTER(C.POINTER(_ProtoResult))]
        L.tsg_proto_result_free.argtypes = [C.POINTER(_ProtoResult)]
        L.tsg_go_parse.argtypes = [C.c_int, C.c_char_p, C.c_size_t, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        L.tsg_write_v2_block.argtypes = [C.c_char_p, vp, C.c_char_p, C.POINTER(C.c_uint64), C.c_size_t, C.c_int,
                                         C.c_char_p, C.c_uint32]
        L.tsg_write_search_block.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int, C.c_uint32]
        L.tsg_fb_search_entry.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.tsg_fb_search_header.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.tsg_synth_search_block.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int, C.c_uint32]
        L.tsg_synth_v2_block.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, vp]
        _lib = L
    return _lib


_shim = None


def shim_pattern_lib():
    """libtsg_shim_pattern.so (built next to libtsg by the same Makefile): the shim's
    per-block call pattern from C threads, for the bench and the coalescer tests."""
    global _shim
    if _shim is None:
        lib()
        path = os.path.join(os.path.dirname(LIB_PATH), "libtsg_shim_pattern.so")
        if not os.path.exists(path):
            raise ImportError(f"libtsg_shim_pattern.so not built at {path}: run __graft_entry__.build()")
        S = C.CDLL(path)
        vp = C.c_void_p
        S.tsgx_shim_pattern.argtypes = [vp, C.POINTER(vp), C.c_size_t, C.c_size_t, C.POINTER(_Query), C.c_uint32,
                                        C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]
        _shim = S
    return _shim


_raw = None


def _raw_lib():
    """A second handle on libtsg whose functions take prebuilt ctypes arguments as-is."""
    global _raw
    if _raw is None:
        lib()
        _raw = C.CDLL(LIB_PATH)
    return _raw


def _check(rc):
    if rc != TSG_OK:
        raise TsgError(rc, lib().tsg_last_error().decode(errors="replace"))


# ---------------------------------------------------------------------------
# request / pipeline

@dataclass
class SearchRequest:
    """tempopb.SearchRequest (pkg/tempopb/tempo.proto:44-52)."""
    tags: Dict[str, str] = field(default_factory=dict)
    min_duration_ms: int = 0
    max_duration_ms: int = 0
    limit: int = 0
    start: int = 0
    end: int = 0

    def _c(self):
        ks = [k.encode() if isinstance(k, str) else k for k in self.tags]
        vs = [v.encode() if isinstance(v, str) else v for v in self.tags.values()]
        n = len(ks)
        r = _Request()
        r.ntags = n
        r._ks = (C.c_char_p * max(n, 1))(*ks)
        r._vs = (C.c_char_p * max(n, 1))(*vs)
        r._kl = (C.c_uint32 * max(n, 1))(*[len(k) for k in ks])
        r._vl = (C.c_uint32 * max(n, 1))(*[len(v) for v in vs])
        r.tag_keys, r.tag_values, r.tag_key_lens, r.tag_value_lens = r._ks, r._vs, r._kl, r._vl
        r.min_duration_ms, r.max_duration_ms = self.min_duration_ms, self.max_duration_ms
        r.limit, r.start, r.end = self.limit, self.start, self.end
        return r


class Pipeline:
    """search.NewSearchPipeline (pipeline.go:26): rewriteTagLookup + ToLower, host side."""

    def __init__(self, req: SearchRequest):
        self.req = req
        self._creq = req._c()
        self.h = C.c_void_p()
        _check(lib().tsg_pipeline_new(C.byref(self._creq), C.byref(self.h)))
        self.query = lib().tsg_pipeline_query(self.h)
        self.query_addr = C.cast(self.query, C.c_void_p).value

    def terms(self):
        q = self.query.contents
        return [(C.string_at(q.keys[i], q.key_lens[i]), C.string_at(q.values[i], q.value_lens[i]))
                for i in range(q.nterms)]

    def matches_block(self, header: bytes) -> bool:
        m = C.c_int()
        _check(lib().tsg_pipeline_matches_header(self.query, header, len(header), C.byref(m)))
        return bool(m.value)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.tsg_pipeline_free(self.h)
            self.h = None


# ---------------------------------------------------------------------------
# results

@dataclass
class TraceSearchMetadata:
    trace_id: bytes          # right-aligned 16 bytes
    trace_id_len: int
    root_service_name: str
    root_trace_name: str
    start_time_unix_nano: int
    duration_ms: int
    end_time_unix_nano: int = 0
    block_idx: int = 0
    entry_idx: int = 0

    @property
    def trace_id_hex(self) -> str:
        """util.TraceIDToHexString: hex, leading zeros trimmed (pkg/util/traceid.go:46-52)."""
        return self.trace_id.hex().lstrip("0")


@dataclass
class SearchMetrics:
    inspected_traces: int
    inspected_bytes: int
    inspected_blocks: int
    skipped_blocks: int
    device_bytes_read: int = 0
    kernel_ns: int = 0
    scan_kernel_ns: int = 0
    scan_bytes: int = 0
    # per block: TSG_OK or the error the reference's Search returns for it after its
    # matches (a damaged data page), with the message
    block_status: List[int] = field(default_factory=list)
    block_errors: List[Optional[str]] = field(default_factory=list)
    skipped_traces: int = 0  # SearchMetrics.SkippedTraces (the proto path's MaxBytes skips; 0 here)
    reruns: int = 0  # extra launches after a record overflow (tsg_metrics.reruns)
    path: int = 0  # PATH_* bits of the kernels that served the search (tsg_metrics.path, ABI 7)


def _unpack(rp) -> (List[TraceSearchMetadata], SearchMetrics):
    r = rp.contents
    out = []
    n = r.n
    if n:
        ids = C.string_at(r.trace_id, 16 * n)
        for i in range(n):
            out.append(TraceSearchMetadata(
                trace_id=ids[16 * i:16 * i + 16], trace_id_len=r.trace_id_len[i],
                root_service_name=C.string_at(r.root_service[i], r.root_service_len[i]).decode(errors="replace"),
                root_trace_name=C.string_at(r.root_name[i], r.root_name_len[i]).decode(errors="replace"),
                start_time_unix_nano=r.start_ns[i], duration_ms=r.duration_ms[i], end_time_unix_nano=r.end_ns[i],
                block_idx=r.block_idx[i], entry_idx=r.entry_idx[i]))
    m = r.metrics
    st = [r.block_status[i] for i in range(r.nblocks)]
    errs = [r.block_error[i].decode(errors="replace") if st[i] else None for i in range(r.nblocks)]
    return out, SearchMetrics(m.traces_inspected, m.bytes_inspected, m.blocks_inspected, m.blocks_skipped,
                              m.device_bytes_read, m.kernel_ns, m.scan_kernel_ns, m.scan_bytes, st, errs,
                              reruns=m.reruns, path=m.path)


# ---------------------------------------------------------------------------
# engine / blocks

class Engine:
    """tsg_ctx: one HIP stream per device. Raises TsgError(TSG_E_DEVICE) without a GPU."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        o = _Options()
        if devices:
            self._devs = (C.c_int32 * len(devices))(*devices)
            o.num_devices, o.devices = len(devices), self._devs
        self.h = C.c_void_p()
        self._raw_calls = {}  # search_raw: prebuilt ctypes arguments (handle values only)
        self._raw_ids = {}  # search_raw fast path for tuple block lists: id -> (tuple, close gen, call)
        # open blocks (weak): closed before tsg_shutdown frees the device contexts they use
        self._open = weakref.WeakSet()
        _check(lib().tsg_init(C.byref(o), C.byref(self.h)))

    @property
    def device_count(self):
        return lib().tsg_device_count(self.h)

    def numa_node(self, dev: int = 0) -> int:
        """NUMA node of the device (tsg_device_numa_node), -1 if unknown."""
        return lib().tsg_device_numa_node(self.h, dev)

    def open_wal_block(self, path: str, device: int = 0) -> "StreamingSearchBlock":
        """Replay a search WAL file (<blockID>:<tenant>:v2:<encoding>[:...]) onto a device."""
        return StreamingSearchBlock(self, path, device)

    def open_block(self, path: str, device: int = 0, pages=None) -> "BackendSearchBlock":
        """A backend search block resident on `device`; pages = (first_page, npages): only that
        page range (tsg_block_open_pages, one shard of a large block)."""
        return BackendSearchBlock(self, path, device, pages=pages)

    def open_live_traces(self, traces: Sequence[Sequence[bytes]], device: int = 0) -> "LiveTraces":
        """A snapshot of the ingester's live traces (each a list of searchData segments, in
        the ingester's iteration order) resident on a device (tsg_live_block_open_mem)."""
        return LiveTraces(self, traces, device)

    def search_tags(self, blocks: Sequence["BackendSearchBlock"]) -> List[bytes]:
        """instance.SearchTags over the blocks (live ones first; tsg_search_tags)."""
        return _packed(lib().tsg_search_tags, _handles(blocks), len(blocks))

    def search_tag_values(self, blocks: Sequence["BackendSearchBlock"], key: bytes, max_bytes: int = -1) -> List[bytes]:
        """instance.SearchTagValues (tsg_search_tag_values): max_bytes = the tenant's
        MaxBytesPerTagValuesQuery (an over-limit set returns []); -1 = no check."""
        key = key.encode() if isinstance(key, str) else key
        return _packed(lib().tsg_search_tag_values, _handles(blocks), len(blocks), key, len(key), max_bytes)

    def search(self, blocks: Sequence["BackendSearchBlock"], pipeline: Pipeline, limit: int = 0, flags: int = 0,
               query_id: int = 0, seen=None):
        """Ordered match sequence + metrics (tsg_search). flags: SEARCH_TIME_*; query_id
        (non-zero) makes the search cancellable with Engine.cancel(query_id); seen: trace IDs
        ((n, 16) uint8, right-aligned) a consumer took before these blocks (they count toward
        the limit)."""
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        opts = _SearchOpts(limit=limit, flags=flags, query_id=query_id)
        seen_arr = _seen(opts, seen)  # noqa: F841  (kept alive across the call)
        rp = C.POINTER(_Result)()
        _check(lib().tsg_search(self.h, arr, len(blocks), pipeline.query, C.byref(opts), C.byref(rp)))
        try:
            return _unpack(rp)
        finally:
            lib().tsg_result_free(rp)

    def search_batch(self, items, depth: int = 0, unpack: bool = True):
        """tsg_search_batch: items = [(blocks, pipeline[, limit]), ...], served back to back (the
        resident kernel takes the next query while earlier ones run). Returns (results, device_ns):
        results[i] = (matches, SearchMetrics) as Engine.search returns them (unpack=False: (match
        count, SearchMetrics)); device_ns = the batch's resident launch's dispatch duration (0 when
        the batch did not run on one resident launch per device)."""
        n = len(items)
        keep = []
        arr = (_SearchItem * max(n, 1))()
        for i, it in enumerate(items):
            blocks, pipeline = it[0], it[1]
            limit = it[2] if len(it) > 2 else 0
            ba = (C.c_void_p * max(len(blocks), 1))(*[b.h.value for b in blocks])
            keep.append(ba)
            arr[i].blocks = C.cast(ba, C.c_void_p).value
            arr[i].nblocks = len(blocks)
            arr[i].query = pipeline.query_addr
            arr[i].opts = _SearchOpts(limit=limit)
        outs = (C.POINTER(_Result) * max(n, 1))()
        dns = C.c_uint64()
        rc = lib().tsg_search_batch(self.h, arr, n, depth, outs, C.byref(dns))
        res = []
        try:
            if rc:
                _check(rc)
            for i in range(n):
                if unpack:
                    res.append(_unpack(outs[i]))
                else:
                    r = outs[i].contents
                    m = r.metrics
                    res.append((r.n, SearchMetrics(m.traces_inspected, m.bytes_inspected, m.blocks_inspected,
                                                   m.blocks_skipped, m.device_bytes_read, m.kernel_ns,
                                                   m.scan_kernel_ns, m.scan_bytes, reruns=m.reruns, path=m.path)))
        finally:
            for i in range(n):
                if outs[i]:
                    lib().tsg_result_free(outs[i])
        return res, dns.value

    def search_raw(self, blocks: Sequence["BackendSearchBlock"], pipeline: Pipeline, limit: int = 0,
                   flags: int = 0, metrics: bool = True):
        """tsg_search without unpacking the matches into Python objects: returns
        (match count, SearchMetrics). The result arrays are assembled by libtsg as
        for any caller (what the Go shim would receive) and then freed. The ctypes
        argument objects are built once per (blocks, pipeline, limit, flags) and kept on
        this Engine (bounded; they hold handle values, not the block objects). A tuple of
        blocks is also looked up by identity (the entry keeps the tuple alive, and any block
        close since the entry was made invalidates it), which skips the per-block key."""
        fast = type(blocks) is tuple
        if fast:
            ik = (id(blocks), pipeline.query_addr, limit, flags)
            ent = self._raw_ids.get(ik)
            if ent is not None and ent[0] is blocks and ent[1] == _block_closes[0]:
                call = ent[2]
            else:
                ent = None
        if not fast or ent is None:
            call = self._raw_call(blocks, pipeline, limit, flags)
            if fast:
                if len(self._raw_ids) >= 64:
                    self._raw_ids.clear()
                self._raw_ids[ik] = (blocks, _block_closes[0], call)
        fn, free, args, rp = call[0], call[1], call[2], call[3]
        rc = fn(*args)
        if rc:
            _check(rc)
        if not metrics:  # (match count only)
            n = rp.contents.n
            free(rp)
            return n, None
        r = rp.contents
        n, m = r.n, r.metrics
        met = SearchMetrics(m.traces_inspected, m.bytes_inspected, m.blocks_inspected, m.blocks_skipped,
                            m.device_bytes_read, m.kernel_ns, m.scan_kernel_ns, m.scan_bytes,
                            reruns=m.reruns, path=m.path)
        free(rp)
        return n, met

    def _raw_call(self, blocks, pipeline, limit, flags):
        key = (pipeline.query_addr, limit, flags) + tuple(b.h.value for b in blocks)
        _cache = self._raw_calls
        call = _cache.get(key)
        if call is None:
            if len(_cache) >= 64:
                _cache.clear()
            L = _raw_lib()  # its own function objects: no argtypes, arguments are prebuilt ctypes objects
            fn, free = L.tsg_search, L.tsg_result_free
            arr = (C.c_void_p * max(len(blocks), 1))(*[b.h.value for b in blocks])
            opts = _SearchOpts(limit=limit, flags=flags)
            rp = C.POINTER(_Result)()
            args = (C.c_void_p(self.h.value), arr, C.c_size_t(len(blocks)), C.c_void_p(pipeline.query_addr),
                    C.byref(opts), C.byref(rp))
            call = _cache[key] = (fn, free, args, rp, arr, opts)
        return call

    def search_columns(self, blocks: Sequence["BackendSearchBlock"], pipeline: Pipeline, limit: int = 0):
        """tsg_search with the ordered matches as numpy columns (large results: no per-record
        Python): dict of trace_id (n, 16) uint8, trace_id_len, start_ns, end_ns, duration_ms,
        block_idx, entry_idx, and root_service / root_name as index arrays into the
        `names` list (distinct strings); plus SearchMetrics."""
        import numpy as np
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        opts = _SearchOpts(limit=limit)
        rp = C.POINTER(_Result)()
        _check(lib().tsg_search(self.h, arr, len(blocks), pipeline.query, C.byref(opts), C.byref(rp)))
        try:
            r = rp.contents
            n = r.n
            cols = {}

            def col(ptr, dt, shape):
                return np.ctypeslib.as_array(ptr, shape).astype(dt) if n else np.zeros(shape, dt)

            cols["trace_id"] = col(r.trace_id, np.uint8, (n, 16)) if n else np.zeros((0, 16), np.uint8)
            cols["trace_id_len"] = col(r.trace_id_len, np.uint8, (n,))
            cols["start_ns"] = col(r.start_ns, np.uint64, (n,))
            cols["end_ns"] = col(r.end_ns, np.uint64, (n,))
            cols["duration_ms"] = col(r.duration_ms, np.uint32, (n,))
            cols["block_idx"] = col(r.block_idx, np.uint32, (n,))
            cols["entry_idx"] = col(r.entry_idx, np.uint64, (n,))
            names, index = [], {}
            arena = C.string_at(r.names, r.names_len) if r.names_len else b""
            for which, off_p, len_p in (("root_service", r.root_service_off, r.root_service_len),
                                        ("root_name", r.root_name_off, r.root_name_len)):
                off = col(off_p, np.uint64, (n,))
                ln = col(len_p, np.uint32, (n,))
                key = (off << np.uint64(32)) | ln.astype(np.uint64)
                uk, inv = np.unique(key, return_inverse=True)
                ids = np.empty(len(uk), np.int64)
                for j, k in enumerate(uk.tolist()):
                    o, l = k >> 32, k & 0xffffffff
                    s = arena[o:o + l] if l else b""
                    ids[j] = index.setdefault(s, len(names))
                    if ids[j] == len(names):
                        names.append(s)
                cols[which] = ids[inv] if n else np.zeros(0, np.int64)
            cols["names"] = names
            m = r.metrics
            met = SearchMetrics(m.traces_inspected, m.bytes_inspected, m.blocks_inspected, m.blocks_skipped,
                                m.device_bytes_read, m.kernel_ns, m.scan_kernel_ns, m.scan_bytes,
                                reruns=m.reruns, path=m.path)
            return cols, met
        finally:
            lib().tsg_result_free(rp)

    def search_wire(self, blocks: Sequence["BackendSearchBlock"], pipeline: Pipeline, limit: int = 0,
                    combine: Optional[int] = None, flags: int = 0, query_id: int = 0, seen=None):
        """tsg_search (+ tsg_results_combine when `combine` is set: instance.Search's
        consumer) packed by tsg_result_pack into a wire buffer (numpy uint8): what a rank
        ships to the merging rank (tempo_amd.shard). No per-record Python."""
        import numpy as np
        if combine is None and seen is None and not query_id:
            # (the search_raw call cache: prebuilt ctypes arguments, no per-call array building)
            fn, free, args, rp = self._raw_call(blocks, pipeline, limit, flags)[:4]
            rc = fn(*args)
            if rc:
                _check(rc)
            try:
                out, ln = C.POINTER(C.c_uint8)(), C.c_size_t()
                _check(lib().tsg_result_pack(rp, C.byref(out), C.byref(ln)))
                try:
                    buf = np.empty(ln.value, np.uint8)
                    C.memmove(buf.ctypes.data, out, ln.value)
                    return buf
                finally:
                    lib().tsg_free(out)
            finally:
                free(rp)
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        opts = _SearchOpts(limit=limit, flags=flags, query_id=query_id)
        seen_arr = _seen(opts, seen)  # noqa: F841
        rp = C.POINTER(_Result)()
        _check(lib().tsg_search(self.h, arr, len(blocks), pipeline.query, C.byref(opts), C.byref(rp)))
        fin = None
        try:
            src = rp
            if combine is not None:
                fin = C.POINTER(_Result)()
                _check(lib().tsg_results_combine(rp, combine, C.byref(fin)))
                src = fin
            out, ln = C.POINTER(C.c_uint8)(), C.c_size_t()
            _check(lib().tsg_result_pack(src, C.byref(out), C.byref(ln)))
            try:
                buf = np.empty(ln.value, np.uint8)
                C.memmove(buf.ctypes.data, out, ln.value)
                return buf
            finally:
                lib().tsg_free(out)
        finally:
            if fin is not None:
                lib().tsg_result_free(fin)
            lib().tsg_result_free(rp)

    def cancel(self, query_id: int):
        """tsg_cancel: the search running (or about to run) with this id stops at its next
        chunk boundary with TSG_E_CANCELLED (the Go shim maps ctx.Done() to this)."""
        _check(lib().tsg_cancel(self.h, query_id))

    def shim_pattern(self, sets: Sequence[Sequence["BackendSearchBlock"]], pipeline: Pipeline, rounds: int,
                     limit: int = 0, digest: bool = False):
        """The Go shim's ingester call pattern (instance_search.go:164-185) driven from C
        threads (libtsg_shim_pattern.so): per query, one thread per block, each a tsg_search
        over its one block with `limit`; query r searches sets[r % len(sets)] (equal-sized
        sets). Returns (per-query wall ns, per-query record counts), and with digest=True
        also the per-query record digests (shim_digest: the sum over the set's blocks of
        FNV-1a 64 over each block's ordered (entry, id, start) records)."""
        sp = shim_pattern_lib()
        nb = len(sets[0])
        assert nb and all(len(s) == nb for s in sets)
        arr = (C.c_void_p * (nb * len(sets)))(*[b.h for s in sets for b in s])
        ns = (C.c_uint64 * rounds)()
        nm = (C.c_uint64 * rounds)()
        dg = (C.c_uint64 * rounds)() if digest else None
        _check(sp.tsgx_shim_pattern(self.h, arr, nb, len(sets), pipeline.query, limit, rounds, ns, nm, dg))
        if digest:
            return list(ns), list(nm), list(dg)
        return list(ns), list(nm)

    def resident_counters(self, dev: int = 0) -> dict:
        """tsg_device_counters: the resident search kernel's launches, queries served, relaunches
        (a launch that left on its idle timeout as a query was posted), quits, slot reads the
        kernel rejected (check mismatch), narrow queries launched plainly because another process
        has a context on the GPU, narrow queries launched plainly (any reason), XCD-split samples."""
        keys = ("launches", "queries", "relaunches", "quits", "rejects", "cotenant_queries", "plain_queries",
                "xsplit_samples")
        buf = (C.c_uint64 * len(keys))()
        _check(lib().tsg_device_counters(self.h, dev, buf, len(keys)))
        return dict(zip(keys, list(buf)))

    def kernel_times(self, cap: int = 65536) -> List[int]:
        """Durations (ns) of the searches run with SEARCH_TIME_DEFER since the last
        call, in launch order (tsg_kernel_times; waits for the device streams)."""
        buf = (C.c_uint64 * cap)()
        n = C.c_size_t()
        _check(lib().tsg_kernel_times(self.h, buf, cap, C.byref(n)))
        return list(buf[:n.value])

    def search_request(self, blocks, req: SearchRequest, limit: Optional[int] = None):
        """instance.Search: ordered matches cut at the limit, then combined + sorted."""
        p = Pipeline(req)
        lim = req.limit if limit is None else limit
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        opts = _SearchOpts(limit=lim)
        rp = C.POINTER(_Result)()
        _check(lib().tsg_search(self.h, arr, len(blocks), p.query, C.byref(opts), C.byref(rp)))
        try:
            fin = C.POINTER(_Result)()
            _check(lib().tsg_results_combine(rp, lim or 20, C.byref(fin)))
            try:
                return _unpack(fin)
            finally:
                lib().tsg_result_free(fin)
        finally:
            lib().tsg_result_free(rp)

    def open_v2block(self, path: str, device: int = 0) -> "V2Block":
        return V2Block(self, path, device)

    def lookup(self, blocks: Sequence["V2Block"], ids, time_start=0, time_end=0, block_start=None,
               block_end=None):
        import numpy as np
        ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 16)
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        o = _LookupOpts(time_start, time_end, block_start, block_end)
        rp = C.POINTER(_LookupResult)()
        _check(lib().tsg_lookup_ids(self.h, arr, len(blocks), ids.ctypes.data, ids.shape[0], C.byref(o),
                                    C.byref(rp)))
        try:
            r = rp.contents
            n = r.n
            if n == 0:
                return np.zeros((0, 5), dtype=np.int64), r.kernel_ns
            cols = [np.ctypeslib.as_array(r.id_idx, (n,)).astype(np.int64),
                    np.ctypeslib.as_array(r.block_idx, (n,)).astype(np.int64),
                    np.ctypeslib.as_array(r.record_idx, (n,)).astype(np.int64),
                    np.ctypeslib.as_array(r.record_start, (n,)).astype(np.int64),
                    np.ctypeslib.as_array(r.record_length, (n,)).astype(np.int64)]
            return np.stack(cols, axis=1), r.kernel_ns
        finally:
            lib().tsg_lookup_result_free(rp)

    def lookup_raw(self, blocks: Sequence["V2Block"], ids) -> Tuple[int, int]:
        """tsg_lookup_ids + tsg_lookup_result_free, nothing converted: (hits, device ns) — what a
        Go caller pays per call (its hit columns are the result's arrays as they are)."""
        import numpy as np
        ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 16)
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        o = _LookupOpts(0, 0, None, None)
        rp = C.POINTER(_LookupResult)()
        _check(lib().tsg_lookup_ids(self.h, arr, len(blocks), ids.ctypes.data, ids.shape[0], C.byref(o),
                                    C.byref(rp)))
        try:
            return int(rp.contents.n), int(rp.contents.kernel_ns)
        finally:
            lib().tsg_lookup_result_free(rp)

    def find(self, blocks: Sequence["V2Block"], ids, time_start=0, time_end=0, block_start=None, block_end=None):
        """tempodb.Find's per-block step on the device (tsg_find_ids): for every lookup hit
        (id_idx, block_idx) the findOne outcome: (id_idx, block_idx, status, object bytes or
        None). status TSG_OK = found, TSG_E_NOT_FOUND = bloom false positive."""
        import numpy as np
        ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 16)
        arr = (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])
        o = _LookupOpts(time_start, time_end, block_start, block_end)
        rp = C.POINTER(_FindResult)()
        _check(lib().tsg_find_ids(self.h, arr, len(blocks), ids.ctypes.data, ids.shape[0], C.byref(o), C.byref(rp)))
        try:
            r = rp.contents
            n = r.n
            total = sum(r.obj_len[i] for i in range(n)) if n else 0
            blob = C.string_at(r.obj_bytes, total) if total else b""
            out = []
            for i in range(n):
                st = r.status[i]
                obj = blob[r.obj_off[i]:r.obj_off[i] + r.obj_len[i]] if st == TSG_OK else None
                out.append((r.id_idx[i], r.block_idx[i], st, obj))
            return out, r.kernel_ns
        finally:
            lib().tsg_find_result_free(rp)

    def open_proto_block(self, path: str, device: int = 0) -> "ProtoBlock":
        return ProtoBlock(self, path, device)

    def proto_search(self, block: "ProtoBlock", tags: Optional[dict] = None, min_ms: int = 0,
                     max_ms: int = 0, start: int = 0, end: int = 0, limit: int = 20,
                     start_page: int = 0, total_pages: int = 0, max_bytes: int = 0,
                     chunk_size_bytes: int = 0) -> ProtoSearchResponse:
        """v2.BackendBlock.Search of one block (tsg_proto_search); raises TsgError where the
        reference's Search returns an error."""
        items = [(k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str) else v)
                 for k, v in (tags or {}).items()]
        n = len(items)
        keys = (C.c_char_p * max(n, 1))(*[k for k, _ in items])
        vals = (C.c_char_p * max(n, 1))(*[v for _, v in items])
        kl = (C.c_uint32 * max(n, 1))(*[len(k) for k, _ in items])
        vl = (C.c_uint32 * max(n, 1))(*[len(v) for _, v in items])
        req = _ProtoRequest(n, keys, kl, vals, vl, min_ms, max_ms, start, end, limit, start_page,
                            total_pages, max_bytes, chunk_size_bytes)
        rp = C.POINTER(_ProtoResult)()
        _check(lib().tsg_proto_search(self.h, block.h, C.byref(req), C.byref(rp)))
        try:
            r = rp.contents
            traces, objs = [], []
            for i in range(r.n):
                tl = r.trace_id_len[i]
                tid = C.string_at(C.addressof(r.trace_ids.contents) + r.trace_id_off[i], tl) if tl else b""
                traces.append(TraceSearchMetadata(
                    trace_id=tid, trace_id_len=tl,
                    root_service_name=C.string_at(r.root_service_name[i], r.root_service_name_len[i]).decode(
                        "utf-8", "surrogateescape"),
                    root_trace_name=C.string_at(r.root_trace_name[i], r.root_trace_name_len[i]).decode(
                        "utf-8", "surrogateescape"),
                    start_time_unix_nano=r.start_time_unix_nano[i], duration_ms=r.duration_ms[i]))
                objs.append(r.object_idx[i])
            return ProtoSearchResponse(traces, r.inspected_traces, r.inspected_bytes, r.skipped_traces, objs,
                                       r.kernel_ns)
        finally:
            lib().tsg_proto_result_free(rp)

    def close(self):
        self._raw_calls = {}
        self._raw_ids = {}
        for b in list(getattr(self, "_open", ())):
            b.close()
        if getattr(self, "h", None) and _lib is not None:
            _lib.tsg_shutdown(self.h)
            self.h = None

    # an engine dropped without close() releases its device contexts when collected (a second
    # context on a device keeps the first one's searches off the resident kernel, pool.hip)
    __del__ = close


_block_closes = [0]  # BackendSearchBlock closes so far


def debug_set(name: str, value: int) -> None:
    """tsg_debug_set: process-wide test hooks ("res_torn": the next `value` resident posts are
    written torn, then repaired)."""
    _check(lib().tsg_debug_set(name.encode(), value))


def _seen(opts, seen):
    """tsg_search_opts.seen_ids / nseen from an (n, 16) uint8 array (returned: keep it alive)."""
    if seen is None or len(seen) == 0:
        return None
    import numpy as np
    arr = np.ascontiguousarray(seen, dtype=np.uint8).reshape(-1, 16)
    opts.seen_ids = arr.ctypes.data
    opts.nseen = arr.shape[0]
    return arr


def _handles(blocks):
    return (C.c_void_p * max(len(blocks), 1))(*[b.h for b in blocks])


def _packed(fn, *args):
    """A packed string list (u32 len + bytes each) from fn(*args, &out, &len, &n)."""
    p, ln, n = C.POINTER(C.c_uint8)(), C.c_size_t(), C.c_size_t()
    _check(fn(*args, C.byref(p), C.byref(ln), C.byref(n)))
    buf = C.string_at(p, ln.value) if ln.value else b""
    lib().tsg_free(p)
    out, o = [], 0
    for _ in range(n.value):
        (l,) = struct.unpack_from("<I", buf, o)
        out.append(buf[o + 4:o + 4 + l])
        o += 4 + l
    return out


class BackendSearchBlock:
    """A backend search block resident on one device (tsg_block)."""

    def __init__(self, eng: Engine, path: str, device: int = 0, _wal: bool = False, _clone_of=None, pages=None):
        self.path = path
        self.pages = pages
        self.h = C.c_void_p()
        if _clone_of is not None:
            _check(lib().tsg_block_clone(eng.h, _clone_of.h, device, C.byref(self.h)))
        elif pages is not None:
            first, n = int(pages[0]), int(pages[1])
            _check(lib().tsg_block_open_pages(eng.h, path.encode(), first, min(n, 2**32 - 1), device,
                                              C.byref(self.h)))
        else:
            opener = lib().tsg_wal_block_open if _wal else lib().tsg_block_open
            _check(opener(eng.h, path.encode(), device, C.byref(self.h)))
        eng._open.add(self)

    def clone(self, eng: Engine, device: int = 0) -> "BackendSearchBlock":
        """tsg_block_clone: a second resident copy (device-to-device), e.g. on another GPU."""
        return BackendSearchBlock(eng, self.path, device, _clone_of=self)

    def info(self):
        i = _BlockInfo()
        _check(lib().tsg_block_info_get(self.h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in _BlockInfo._fields_}

    def _strings(self, fn, *args):
        return _packed(fn, self.h, *args)

    def tags(self):
        return self._strings(lib().tsg_block_tags)

    def tag_values(self, key: bytes):
        return self._strings(lib().tsg_block_tag_values, key, len(key))

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _block_closes[0] += 1  # (search_raw's identity cache entries made before this are stale)
            _lib.tsg_block_close(self.h)
            self.h = None

    __del__ = close


class StreamingSearchBlock(BackendSearchBlock):
    """A search WAL file replayed into a resident block (tsg_wal_block_open): the
    StreamingSearchBlock of search.RescanBlocks, searched through the same tsg_search."""

    def __init__(self, eng: Engine, path: str, device: int = 0):
        super().__init__(eng, path, device, _wal=True)


def live_wire(traces: Sequence[Sequence[bytes]]):
    """[[segment, ...] per trace] -> (bytes, seg_off u64[nsegs + 1], trace_seg u64[ntraces + 1])."""
    import numpy as np
    segs = [sg for t in traces for sg in t]
    seg_off = np.zeros(len(segs) + 1, dtype=np.uint64)
    if segs:
        seg_off[1:] = np.cumsum([len(sg) for sg in segs])
    trace_seg = np.zeros(len(traces) + 1, dtype=np.uint64)
    if len(traces):
        trace_seg[1:] = np.cumsum([len(t) for t in traces])
    return b"".join(segs), seg_off, trace_seg


class LiveTraces(BackendSearchBlock):
    """The ingester's live traces (instance.searchLiveTraces, modules/ingester/
    instance_search.go:83-130) as one resident block: a row per searchData segment;
    tsg_search matches each segment and combines a trace's matches into one result."""

    def __init__(self, eng: Engine, traces: Sequence[Sequence[bytes]], device: int = 0):
        self.path = None
        self.h = C.c_void_p()
        data, seg_off, trace_seg = live_wire(traces)
        _check(lib().tsg_live_block_open_mem(eng.h, data, seg_off.ctypes.data, len(seg_off) - 1,
                                             trace_seg.ctypes.data, len(trace_seg) - 1, device, C.byref(self.h)))
        eng._open.add(self)


@dataclass
class ProtoSearchResponse:
    """tempopb.SearchResponse of one v2.BackendBlock.Search (traces in object order)."""
    traces: List[TraceSearchMetadata]
    inspected_traces: int
    inspected_bytes: int
    skipped_traces: int
    object_idx: List[int]
    kernel_ns: int = 0


class ProtoBlock:
    """A v2 trace block whose objects are trace protos (tsg_proto_block), resident on one
    device: the querier's SearchBlock path (tempodb.Search -> BackendBlock.Search)."""

    def __init__(self, eng: Engine, path: str, device: int = 0):
        self.path = path
        self.h = C.c_void_p()
        _check(lib().tsg_proto_block_open(eng.h, path.encode(), device, C.byref(self.h)))
        eng._open.add(self)

    def info(self) -> dict:
        o = (C.c_uint64 * 4)()
        _check(lib().tsg_proto_block_info(self.h, o))
        return {"objects": o[0], "pages": o[1], "keys": o[2], "device_bytes": o[3]}

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.tsg_proto_block_close(self.h)
            self.h = None

    __del__ = close


class V2Block:
    def __init__(self, eng: Engine, path: str, device: int = 0):
        self.h = C.c_void_p()
        _check(lib().tsg_v2block_open(eng.h, path.encode(), device, C.byref(self.h)))
        eng._open.add(self)

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.tsg_v2block_close(self.h)
            self.h = None

    __del__ = close


# ---------------------------------------------------------------------------
# writer tooling (host)

def encode_entries(entries: Iterable[dict]) -> bytes:
    """Entry list wire format of tsg_write_search_block.

    entry = {"id": bytes, "start": int, "end": int, "tags": {key: [values]}}"""
    out = bytearray()
    for e in entries:
        tid = e["id"]
        out += struct.pack("<I", len(tid)) + tid
        pairs = []
        for k, vs in e.get("tags", {}).items():
            if isinstance(vs, (str, bytes)):
                vs = [vs]
            for v in vs:
                pairs.append((k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str) else v))
        out += struct.pack("<QQI", e.get("start", 0) & (2**64 - 1), e.get("end", 0) & (2**64 - 1), len(pairs))
        for k, v in pairs:
            out += struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v
    return bytes(out)


def write_search_block(path: str, entries: Iterable[dict], encoding: int = ENC_SNAPPY, page_size: int = 0):
    buf = encode_entries(entries)
    _check(lib().tsg_write_search_block(path.encode(), buf, len(buf), encoding, page_size))


def write_wal_search(path: str, entries: Iterable[dict], encoding: int = ENC_SNAPPY):
    """StreamingSearchBlock.Append of each entry, in order, into a search WAL file."""
    buf = encode_entries(entries)
    _check(lib().tsg_write_wal_search(path.encode(), buf, len(buf), encoding))


def wal_filename(encoding: int = ENC_SNAPPY, block_id: str = "1c505e8b-26cd-4621-ba7d-792bb55282d5",
                 tenant: str = "single-tenant") -> str:
    """<blockID>:<tenant>:v2:<encoding>: (the name wal.ParseFilename reads)."""
    return f"{block_id}:{tenant}:v2:{ENC_NAMES[encoding]}:"


def _bytes_out(fn, *args):
    p, n = C.POINTER(C.c_uint8)(), C.c_size_t()
    _check(fn(*args, C.byref(p), C.byref(n)))
    b = C.string_at(p, n.value)
    lib().tsg_free(p)
    return b


def fb_search_entry(entry: dict) -> bytes:
    """SearchEntryMutable.ToBytes (pkg/tempofb/search_entry_mutable.go:41-46)."""
    buf = encode_entries([entry])
    return _bytes_out(lib().tsg_fb_search_entry, buf, len(buf))


def fb_search_header(entries: Iterable[dict]) -> bytes:
    """SearchBlockHeaderMutable.ToBytes after AddEntry of each entry."""
    buf = encode_entries(entries)
    return _bytes_out(lib().tsg_fb_search_header, buf, len(buf))


def synth_search_block(path: str, n: int, seed: int = 0, profile: int = 0, encoding: int = ENC_SNAPPY,
                       page_size: int = 1024 * 1024):
    _check(lib().tsg_synth_search_block(path.encode(), n, seed, profile, encoding, page_size))


def write_v2_block(path: str, ids, objects: Sequence[bytes], encoding: int = 0, data_encoding: str = "v2",
                   index_downsample_bytes: int = 0):
    """tsg_write_v2_block: a v2 block of the given objects (ids: (n, 16) uint8, ascending)."""
    import numpy as np
    ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 16)
    blob = b"".join(objects)
    off = [0]
    for o in objects:
        off.append(off[-1] + len(o))
    offs = (C.c_uint64 * len(off))(*off)
    _check(lib().tsg_write_v2_block(path.encode(), ids.ctypes.data, blob, offs, ids.shape[0], encoding,
                                    data_encoding.encode(), index_downsample_bytes))


def go_parse(kind: str, s) -> tuple:
    """Go strconv as the engine implements it: kind "int" | "float" | "bool" -> (ok, value)."""
    b = s.encode() if isinstance(s, str) else s
    f, i = C.c_double(), C.c_int64()
    k = {"int": 0, "float": 1, "bool": 2}[kind]
    ok = lib().tsg_go_parse(k, b, len(b), C.byref(f), C.byref(i))
    if ok < 0:
        raise ValueError(kind)
    return bool(ok), (f.value if kind == "float" else (bool(i.value) if kind == "bool" else i.value))


def synth_v2_block(path: str, n: int, seed: int = 0):
    import numpy as np
    ids = np.zeros((n, 16), dtype=np.uint8)
    _check(lib().tsg_synth_v2_block(path.encode(), n, seed, ids.ctypes.data))
    return ids
