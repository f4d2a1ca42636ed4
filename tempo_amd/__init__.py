"""tempo_amd — MI355X-native engine for Tempo's backend trace search path.

The product is libtsg.so (C ABI, include/tsg.h): HIP kernels for gfx950 behind
the drop-in boundary of tempodb/search BackendSearchBlock.Search and the v2
bloom/index trace-ID lookup (+ device findOne), and the proto-object
BackendBlock.Search. ``tempo_amd.tsg`` is the ctypes host mirror.
"""
from .tsg import (  # noqa: F401
    BackendSearchBlock, Engine, StreamingSearchBlock, LiveTraces, live_wire, Pipeline, SearchMetrics, SearchRequest, TraceSearchMetadata, TsgError, V2Block,
    ENC_NONE, ENC_SNAPPY, SEARCH_TIME_ALL, SEARCH_TIME_DEFER, SEARCH_TIME_SCAN, fb_search_entry, fb_search_header, lib, synth_search_block, synth_v2_block,
    write_search_block, write_wal_search, wal_filename, ProtoBlock, ProtoSearchResponse, write_v2_block, go_parse,
    TSG_OK, TSG_E_NOT_FOUND, TSG_E_CORRUPT, TSG_E_UNSUPPORTED_ENCODING, TSG_E_DEVICE, TSG_E_CANCELLED, TSG_E_OOM,
    TSG_E_INVALID, TSG_E_UNSUPPORTED, TSG_E_IO, PATH_RESIDENT, PATH_PLAIN, PATH_OTHER, PATH_COTENANT, debug_set,
)
