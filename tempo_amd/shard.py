"""Multi-GPU search: block sharding over ranks and the frontend's response merge.

One process per GPU. The search path partitions by block (the frontend shards a
query into per-block jobs, modules/frontend/searchsharding.go:325-367), so each
rank searches only its own resident blocks with no data-path collective. The one
exchange is the final gather of per-rank responses to rank 0, which then merges
them the way the frontend's `searchResponse` does (searchsharding.go:32-125):

* `addResponse` (searchsharding.go:71-86): traces keyed by trace ID, first one
  seen wins (no CombineSearchResults here); InspectedBytes / InspectedTraces /
  SkippedBlocks / SkippedTraces summed; InspectedBlocks is set by the sharder to
  the number of blocks in the query (searchsharding.go:221), not summed.
* `shouldQuit` (searchsharding.go:88-105): stop taking responses once the map
  holds more than `limit` traces (or a job failed: `on_error="raise"`).
* `result` (searchsharding.go:107-125): traces sorted by start time descending.

The reference consumes job responses in completion order (racy); here they are
consumed in rank order and ties keep first-seen order, which makes the merged
response deterministic.

Responses travel packed ("wire" buffers, include/tsg.h): 40-byte
TraceSearchMetadata records, the names as a per-response table, the metrics and
every block's status and error. A rank packs its tsg_result in libtsg
(`Engine.search_wire`, tsg_result_pack), the wires are gathered as byte tensors
(`dist.gather`: RCCL over xGMI on the GPUs, gloo on the CPU) and rank 0 merges
them in libtsg (tsg_wire_merge: parallel hash-partitioned first-wins dedupe +
radix sort by start time); numpy views read the merged buffer. No per-record
Python on the path.

Trace-ID lookup shards the probe ids instead (bloom + index replicated on every
rank, tempodb.Find's fan-out over blocks stays rank-local): `shard_ids` gives each
rank a contiguous id slice and `distributed_lookup` gathers the per-rank hit
tables (int64 rows id, block, record, start, length); concatenated in rank order
they are already sorted by (id, block).
"""
import ctypes as C
import struct
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .tsg import TSG_E_INVALID, SearchMetrics, TraceSearchMetadata, TsgError, _check, lib

WIRE_MAGIC = 0x57475354
WIRE_VERSION = 1
_HDR = struct.Struct("<II5Q5QQ")  # tsg_wire_header
assert _HDR.size == 96
REC_DTYPE = np.dtype([("trace_id", "V16"), ("start_ns", "<u8"), ("duration_ms", "<u4"), ("root_service", "<u4"),
                      ("root_name", "<u4"), ("trace_id_len", "u1"), ("pad", "V3")])  # tsg_trace_rec
assert REC_DTYPE.itemsize == 40


def shard_range(n_blocks: int, world: int, rank: int) -> range:
    """Contiguous block range owned by `rank` (blocks keep their global order)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return range(n_blocks * rank // world, n_blocks * (rank + 1) // world)


@dataclass(frozen=True)
class Part:
    """One rank's piece of a query's block list: block `block` (its index in the list) whole
    (npages == 0), or its index records [first_page, first_page + npages)."""
    block: int
    first_page: int = 0
    npages: int = 0

    @property
    def whole(self) -> bool:
        return self.npages == 0

    def pages(self):
        """(first_page, npages) for Engine.open_block(pages=...) / oracle.Block(pages=...), or None."""
        return None if self.whole else (self.first_page, self.npages)


def block_sizes(paths: Sequence[str]) -> Tuple[List[int], List[int]]:
    """(bytes, pages) of each search block directory: the size of its `search` file and the
    index records its search.meta.json declares (0, 0 when the block has no search data: a
    no-op for Search). The frontend sizes jobs the same way: bytes per page = size / records
    (modules/frontend/searchsharding.go:331-339)."""
    import json
    import os
    sizes, pages = [], []
    for p in paths:
        try:
            with open(os.path.join(p, "search.meta.json")) as f:
                n = int(json.load(f).get("indexRecords", 0))
            sz = os.path.getsize(os.path.join(p, "search"))
        except (OSError, ValueError):
            n, sz = 0, 0
        sizes.append(sz if n else 0)
        pages.append(n)
    return sizes, pages


def plan_shards(sizes: Sequence[int], pages: Sequence[int], world: int, split: bool = True) -> List[List[Part]]:
    """Size-balanced shards of a query's blocks over `world` ranks: rank r
    takes a contiguous stretch of the blocks in query order — rank order stays block order,
    which the frontend merge's tie order and the limit protocol (distributed_search_limit)
    rely on — ending where the cumulative bytes reach (r + 1) / world of the total. A cut that
    falls inside a block splits it at the page boundary nearest the cut (split=True: pages of
    size / records bytes, the frontend's estimate, searchsharding.go:331-339, so one giant
    block is spread over several ranks); with split=False the cut moves to the nearer block
    boundary (whole blocks only). Every page of every block lands in exactly one part."""
    if world <= 0:
        raise ValueError(f"bad world {world}")
    nb = len(sizes)
    if len(pages) != nb:
        raise ValueError("sizes and pages differ in length")
    cum = [0]
    for sz in sizes:
        cum.append(cum[-1] + max(0, int(sz)))
    total = cum[-1]
    # cut r (1 <= r < world) as a position (block, page): everything before it goes to ranks < r
    cuts = [(0, 0)]
    for r in range(1, world):
        c = total * r / world
        b = 0
        while b < nb and cum[b + 1] <= c:
            b += 1
        if b >= nb:
            pos = (nb, 0)
        else:
            if split and pages[b] > 1 and sizes[b] > 0:
                k = int(round((c - cum[b]) / (sizes[b] / pages[b])))
                k = min(max(k, 0), pages[b])
            else:
                k = 0 if c - cum[b] <= cum[b + 1] - c else pages[b]
            pos = (b, k) if k < pages[b] else (b + 1, 0)
        cuts.append(max(pos, cuts[-1]))
    cuts.append((nb, 0))
    out = []
    for r in range(world):
        (b0, p0), (b1, p1) = cuts[r], cuts[r + 1]
        parts = []
        for b in range(b0, min(b1 + 1, nb)):
            lo = p0 if b == b0 else 0
            hi = p1 if b == b1 else pages[b]
            if b == b1 and p1 == 0:
                break
            if lo == 0 and hi >= pages[b]:
                parts.append(Part(b))
            elif hi > lo:
                parts.append(Part(b, lo, hi - lo))
        out.append(parts)
    return out


def _pad8(x):
    return (x + 7) & ~7


@dataclass
class Response:
    """A tempopb.SearchResponse in columns: `recs` (REC_DTYPE), the name table
    (`names[name_off[k]:name_off[k+1]]`), the metrics and every block's status."""
    recs: np.ndarray
    name_off: np.ndarray
    names: bytes
    metrics: SearchMetrics
    block_status: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    block_errors: List[Optional[str]] = field(default_factory=list)

    def __len__(self):
        return len(self.recs)

    def name(self, k: int) -> str:
        return self.names[int(self.name_off[k]):int(self.name_off[k + 1])].decode(errors="replace")

    def traces(self) -> List[TraceSearchMetadata]:
        """The records as TraceSearchMetadata objects (for small responses)."""
        r = self.recs
        return [TraceSearchMetadata(trace_id=bytes(r["trace_id"][i]), trace_id_len=int(r["trace_id_len"][i]),
                                    root_service_name=self.name(r["root_service"][i]),
                                    root_trace_name=self.name(r["root_name"][i]),
                                    start_time_unix_nano=int(r["start_ns"][i]), duration_ms=int(r["duration_ms"][i]))
                for i in range(len(r))]

    def hex_ids(self) -> List[str]:
        """util.TraceIDToHexString of every record (pkg/util/traceid.go:46-52)."""
        return [bytes(x).hex().lstrip("0") for x in self.recs["trace_id"]]


def response_from_traces(traces: Sequence[TraceSearchMetadata], metrics: SearchMetrics) -> Response:
    """A Response from TraceSearchMetadata objects (test stand-ins, small lists)."""
    table = {"": 0}
    recs = np.zeros(len(traces), REC_DTYPE)
    for i, t in enumerate(traces):
        s = table.setdefault(t.root_service_name, len(table))
        n = table.setdefault(t.root_trace_name, len(table))
        recs[i] = (bytes(t.trace_id).rjust(16, b"\0")[-16:], t.start_time_unix_nano, t.duration_ms, s, n,
                   t.trace_id_len, b"\0\0\0")
    enc = [k.encode() for k in table]
    off = np.zeros(len(enc) + 1, np.uint32)
    off[1:] = np.cumsum([len(b) for b in enc]) if enc else []
    st = np.asarray(metrics.block_status or [], np.int32)
    errs = list(metrics.block_errors or [None] * len(st))
    return Response(recs, off, b"".join(enc), metrics, st, errs)


def to_wire(resp: Response) -> np.ndarray:
    """Response -> wire buffer (uint8 array), numpy only."""
    n, nn, nl = len(resp.recs), len(resp.name_off) - 1, len(resp.names)
    st = np.asarray(resp.block_status, np.int32)
    err = b"".join(struct.pack("<I", len(e.encode())) + e.encode() for s, e in zip(st, resp.block_errors) if s)
    size = _HDR.size + _pad8(40 * n) + _pad8(4 * (nn + 1)) + _pad8(nl) + _pad8(4 * len(st)) + _pad8(len(err))
    buf = np.empty(size, np.uint8)
    m = resp.metrics
    _HDR.pack_into(buf, 0, WIRE_MAGIC, WIRE_VERSION, n, nn, nl, len(st), len(err), m.inspected_traces,
                   m.inspected_bytes, m.inspected_blocks, m.skipped_blocks, m.skipped_traces, 0)
    o = _HDR.size
    for part in (np.ascontiguousarray(resp.recs, REC_DTYPE).view(np.uint8).reshape(-1),
                 np.ascontiguousarray(resp.name_off, np.uint32).view(np.uint8), np.frombuffer(resp.names, np.uint8),
                 st.view(np.uint8), np.frombuffer(err, np.uint8)):
        buf[o:o + part.size] = part
        buf[o + part.size:o + _pad8(part.size)] = 0
        o += _pad8(part.size)
    return buf


def from_wire(buf) -> Response:
    """Wire buffer -> Response (numpy views into `buf` where possible)."""
    b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8).reshape(-1)
    (magic, ver, n, nn, nl, nb, el, it, ib, ibl, sb, skt, _) = _HDR.unpack_from(b, 0)
    if magic != WIRE_MAGIC or ver != WIRE_VERSION:
        raise ValueError("not a tsg wire buffer")
    o = _HDR.size
    recs = b[o:o + 40 * n].view(REC_DTYPE)
    o += _pad8(40 * n)
    off = b[o:o + 4 * (nn + 1)].view(np.uint32)
    o += _pad8(4 * (nn + 1))
    names = b[o:o + nl].tobytes()
    o += _pad8(nl)
    st = b[o:o + 4 * nb].view(np.int32)
    o += _pad8(4 * nb)
    eb = b[o:o + el].tobytes()
    errs, e = [], 0
    for s in st:
        if s:
            (k,) = struct.unpack_from("<I", eb, e)
            errs.append(eb[e + 4:e + 4 + k].decode(errors="replace"))
            e += 4 + k
        else:
            errs.append(None)
    met = SearchMetrics(it, ib, ibl, sb, block_status=st.tolist(), block_errors=errs, skipped_traces=skt)
    return Response(recs, off, names, met, st, errs)


def _as_bytes_ptr(w):
    a = np.ascontiguousarray(np.frombuffer(w, np.uint8) if not isinstance(w, np.ndarray) else w.view(np.uint8))
    return a, a.ctypes.data_as(C.POINTER(C.c_uint8))


def merge_wires(wires: Sequence, limit: int, total_blocks: int, out: Optional[np.ndarray] = None) -> Response:
    """The frontend merge (tsg_wire_merge) of wire responses in order -> merged Response.
    `out`: a caller-owned uint8 buffer to merge into (reused across queries: no allocation
    and no page faults per merge; the Response's arrays are views into it); grown if short."""
    keep = [_as_bytes_ptr(w) for w in wires]
    n = len(keep)
    ptrs = (C.POINTER(C.c_uint8) * max(n, 1))(*[p for _, p in keep])
    lens = (C.c_size_t * max(n, 1))(*[a.size for a, _ in keep])
    # the merged wire is never longer than its inputs; with none it is the header + one name offset
    need = max(_HDR.size + 8, sum(a.size for a, _ in keep))
    if out is None or out.size < need:
        out = np.empty(need, np.uint8)
    ln = C.c_size_t()
    lim = min(int(limit), 2**64 - 1)
    rc = lib().tsg_wire_merge(ptrs, lens, n, lim, total_blocks, out.ctypes.data, out.size, C.byref(ln))
    if rc == TSG_E_INVALID and ln.value > out.size:  # (short buffer: the library reports the size)
        out = np.empty(ln.value, np.uint8)
        rc = lib().tsg_wire_merge(ptrs, lens, n, lim, total_blocks, out.ctypes.data, out.size, C.byref(ln))
    _check(rc)
    return from_wire(out[:ln.value])


def _raise_first_error(resp: Response):
    for s, e in zip(resp.block_status, resp.block_errors):
        if s:
            raise TsgError(int(s), e or "search job failed")


def merge_responses(responses: Sequence[Tuple[Sequence[TraceSearchMetadata], SearchMetrics]],
                    limit: int, total_blocks: int, on_error: str = "keep"
                    ) -> Tuple[List[TraceSearchMetadata], SearchMetrics]:
    """Frontend merge of per-shard (traces, metrics) responses, in shard order.

    on_error: "keep" returns every block's status / error in the metrics (the ingester logs
    a failed block and keeps the others' results, instance_search.go:179-182); "raise"
    raises the first one, as a failed job does to the frontend request (setError ->
    shouldQuit, searchsharding.go:64-69,88-94)."""
    merged = merge_wires([to_wire(response_from_traces(t, m)) for t, m in responses], limit, total_blocks)
    if on_error == "raise":
        _raise_first_error(merged)
    return merged.traces(), merged.metrics


def distributed_search(search_local: Callable[[], Tuple[List[TraceSearchMetadata], SearchMetrics]],
                       limit: int, total_blocks: int, group=None, dst: int = 0, on_error: str = "keep"
                       ) -> Optional[Tuple[List[TraceSearchMetadata], SearchMetrics]]:
    """Run this rank's search, gather the responses on `dst` (pickled: gather_object,
    fine for limit-bounded responses), merge there. Returns the merged response on `dst`,
    None elsewhere. Works on any torch.distributed backend."""
    import torch.distributed as dist
    mine = search_local()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    got = [None] * world if rank == dst else None
    dist.gather_object(mine, got, dst=dst, group=group)
    if rank != dst:
        return None
    return merge_responses(got, limit, total_blocks, on_error)


_GATHER_CACHE = {}  # (device, slot, role) -> grow-only 1-D uint8 tensors reused across gathers


def _cached(device, slot, width):
    import torch
    key = (str(device), slot)
    t = _GATHER_CACHE.get(key)
    if t is None or t.numel() < width:
        t = torch.empty(max(width, 1), dtype=torch.uint8, device=device)
        _GATHER_CACHE[key] = t
    return t[:width]


def _gather_bytes(parts: Sequence, device, group, dst):
    """Gather variable-length byte buffers (one list per rank) to `dst` as tensors: sizes
    first, then every part padded to the longest of any rank. The send and receive tensors
    are kept between calls (a query's gather then allocates nothing and takes no page faults);
    a numpy part that is already that long is sent without a copy."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    arrs = [p if isinstance(p, np.ndarray) else np.frombuffer(bytearray(p), np.uint8) for p in parts]
    sizes = torch.tensor([a.size for a in arrs], dtype=torch.int64, device=device)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)] if rank == dst else None
    dist.gather(sizes, all_sizes, dst=dst, group=group)
    mx = sizes.max().clone() if arrs else torch.zeros((), dtype=torch.int64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    width = max(1, int(mx.item()))
    result = [] if rank == dst else None
    for i, a in enumerate(arrs):
        if a.size == width and a.flags.writeable and a.flags.c_contiguous and str(device) == "cpu":
            t = torch.from_numpy(a)
        else:
            t = _cached(device, ("send", i), width)
            if a.size:
                t[:a.size].copy_(torch.from_numpy(np.ascontiguousarray(a)))
            if a.size < width:
                t[a.size:].zero_()
        recv = [_cached(device, ("recv", i, r), width) for r in range(world)] if rank == dst else None
        dist.gather(t, recv, dst=dst, group=group)
        if rank == dst:
            result.append(recv)
    if rank != dst:
        return None
    out = []
    for r in range(world):
        sz = all_sizes[r].cpu().tolist()
        out.append([result[i][r][:sz[i]].cpu().numpy() for i in range(len(arrs))])
    return out


WireSource = Union[bytes, np.ndarray, Response, Tuple[Sequence[TraceSearchMetadata], SearchMetrics]]


def _wire_of(x: WireSource) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return x.view(np.uint8).reshape(-1)
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytearray(x), np.uint8)
    if isinstance(x, Response):
        return to_wire(x)
    traces, met = x
    return to_wire(response_from_traces(traces, met))


def distributed_search_packed(search_local: Callable[[], WireSource], limit: int, total_blocks: int, device=None,
                              group=None, dst: int = 0, on_error: str = "keep", columns: bool = False):
    """`distributed_search` with the responses moved as wire buffers (byte tensors on
    `device`: a CUDA device with the nccl backend = RCCL over xGMI; the CPU with gloo) and
    merged in libtsg. `search_local` returns this rank's response: a wire buffer
    (`Engine.search_wire`), a Response, or (traces, metrics). On `dst`: the merged
    response as (traces, metrics), or the Response with columns=True; None elsewhere."""
    import torch.distributed as dist
    wire = _wire_of(search_local())
    got = _gather_bytes([wire], device or "cpu", group, dst)
    if dist.get_rank(group) != dst:
        return None
    merged = merge_wires([g[0] for g in got], limit, total_blocks)
    if on_error == "raise":
        _raise_first_error(merged)
    return merged if columns else (merged.traces(), merged.metrics)


class ShmGather:
    """The frontend merge for the ranks of one node through shared memory (tsg_shm_*, DESIGN.md
    §5): each rank puts its wire response for a query into its slot of /dev/shm/<name>, rank 0
    merges every rank's slot in place when all have answered (no collective, no copy into a
    tensor). Queries are numbered 1, 2, ... in call order on every rank; a rank may put query
    s + 1 while rank 0 merges s (double-buffered slots). Rank 0 creates the file (reset) before
    the others open it: `group` (a torch.distributed group of the node's ranks) orders that.
    A response larger than `slot_bytes` fails its put (TSG_E_INVALID): gather it another way."""

    def __init__(self, name: str, world: int, rank: int, group=None, slot_bytes: int = 16 << 20):
        import torch.distributed as dist
        self.world, self.rank, self.slot_bytes, self.seq = world, rank, slot_bytes, 0
        self.h = C.c_void_p()
        self._out = None
        if rank == 0:
            _check(lib().tsg_shm_open(name.encode(), world, rank, slot_bytes, 1, C.byref(self.h)))
        dist.barrier(group=group)
        if rank != 0:
            _check(lib().tsg_shm_open(name.encode(), world, rank, slot_bytes, 0, C.byref(self.h)))
        dist.barrier(group=group)

    def query(self, wire, limit: int, total_blocks: int, timeout_s: float = 60.0) -> Optional["Response"]:
        """Put this rank's wire for the next query; on rank 0 return the merged Response."""
        self.seq = self.seq + 1 if self.seq < 0xFFFFFFFF else 1
        w = _wire_of(wire)
        _check(lib().tsg_shm_put(self.h, self.seq, w.ctypes.data, w.size, timeout_s))
        if self.rank != 0:
            return None
        if self._out is None:
            self._out = np.empty(self.world * self.slot_bytes + 4096, np.uint8)
        ln = C.c_size_t()
        lim = min(int(limit), 2**64 - 1)
        _check(lib().tsg_shm_merge(self.h, self.seq, lim, total_blocks, self._out.ctypes.data, self._out.size,
                                   C.byref(ln), timeout_s))
        return from_wire(self._out[:ln.value])

    def close(self):
        if self.h:
            lib().tsg_shm_close(self.h)
            self.h = C.c_void_p()


def shard_ids(n_ids: int, world: int, rank: int) -> range:
    """Contiguous probe-id slice owned by `rank` (config 5: 10 M ids over the GPUs)."""
    return shard_range(n_ids, world, rank)


def distributed_lookup(lookup_local: Callable[[object], object], ids, device=None, group=None, dst: int = 0):
    """Each rank looks up its id slice against every (replicated) block; rank `dst`
    returns the global hit table (int64 rows: id, block, record, start, length) sorted
    by (id, block), others None. `lookup_local(id_slice)` returns the rank's table with
    slice-local id indices (e.g. `lambda x: engine.lookup(blocks, x)[0]`)."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sl = shard_ids(len(ids), world, rank)
    hits = np.asarray(lookup_local(ids[sl.start:sl.stop]), dtype=np.int64).reshape(-1, 5).copy()
    hits[:, 0] += sl.start
    got = _gather_bytes([hits.view(np.uint8).reshape(-1)], device or "cpu", group, dst)
    if rank != dst:
        return None
    return np.concatenate([np.frombuffer(g[0].tobytes(), dtype=np.int64).reshape(-1, 5) for g in got])


# ---------------------------------------------------------------------------
# limit queries over ranks: the consumer's early exit across the block shards

def _distinct_in_order(resp: Response) -> np.ndarray:
    """The response's trace IDs, each once, in first-occurrence order ((k, 16) uint8)."""
    if len(resp.recs) == 0:
        return np.zeros((0, 16), np.uint8)
    ids = np.ascontiguousarray(resp.recs["trace_id"]).view(np.uint8).reshape(-1, 16)
    _, first = np.unique(ids, axis=0, return_index=True)
    return ids[np.sort(first)]


def concat_responses(resps: Sequence[Response]) -> Response:
    """Responses of consecutive block ranges as one: records one after another (names
    re-indexed into one table), metrics summed, block statuses concatenated."""
    recs, offs, names, st, errs = [], [np.zeros(1, np.uint32)], [], [], []
    nn = nb = 0
    m = SearchMetrics(0, 0, 0, 0)
    for r in resps:
        x = np.array(r.recs, copy=True)
        x["root_service"] += nn
        x["root_name"] += nn
        recs.append(x)
        offs.append(np.asarray(r.name_off[1:], np.uint64) + nb)
        names.append(r.names)
        nn += len(r.name_off) - 1
        nb += len(r.names)
        m.inspected_traces += r.metrics.inspected_traces
        m.inspected_bytes += r.metrics.inspected_bytes
        m.inspected_blocks += r.metrics.inspected_blocks
        m.skipped_blocks += r.metrics.skipped_blocks
        m.skipped_traces += r.metrics.skipped_traces
        st.append(np.asarray(r.block_status, np.int32))
        errs.extend(r.block_errors)
    status = np.concatenate(st) if st else np.zeros(0, np.int32)
    m.block_status, m.block_errors = status.tolist(), errs
    return Response(np.concatenate(recs) if recs else np.zeros(0, REC_DTYPE),
                    np.concatenate(offs).astype(np.uint32), b"".join(names), m, status, errs)


_CTRL_KEEP, _CTRL_SEEDED, _CTRL_DROP = 0, 1, 2


def distributed_search_limit(search, cancel, limit: int, group=None, dst: int = 0,
                             query_id: int = 0) -> Optional[Response]:
    """A limit-L search over block shards (rank r holds the r-th range of the query's blocks,
    in block order) that returns on `dst` exactly what one consumer over all blocks in order
    returns — instance.Search's consumer (instance_search.go:45-60) stopping at the L-th
    distinct trace ID, records in order, metrics of the blocks and pages it reached — while
    later ranks stop early (ranks publish what they matched, the host finds
    the prefix that holds L distinct IDs, the rest is cancelled; the frontend's shouldQuit,
    modules/frontend/searchsharding.go:88-106).

    search(seen, qid) -> wire: this rank's tsg_search over its blocks with limit L (e.g.
    Engine.search_wire(blocks, pipe, limit=L, query_id=qid, seen=seen)); seen = trace IDs
    taken before these blocks, or None. cancel(qid): Engine.cancel.

    1. Every rank searches its shard with limit L at once (its own early exit).
    2. `dst` takes the ranks' reports in rank order and runs the consumer over their
       distinct IDs. Ranks before the one where it reaches L keep their result (they did not
       reach L alone, so they hold every match); that rank (r*) searches again with the IDs
       before it as `seen` (unless none), stopping exactly where the single consumer stops;
       ranks after it are told to drop, cancelling a search still running (tsg_cancel).
    3. The kept responses are gathered to `dst` and concatenated in rank order.
    Messages are point-to-point over `group` (gloo: host tensors). limit <= 0 means every
    match, as in tsg_search: no rank is a stop point, every response is kept."""
    import threading

    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gdst = dst if group is None else dist.get_global_rank(group, dst)

    def grank(r):
        return r if group is None else dist.get_global_rank(group, r)

    def send_ids(ids, to):
        dist.send(torch.tensor([len(ids)], dtype=torch.int64), grank(to), group=group)
        if len(ids):
            dist.send(torch.from_numpy(np.ascontiguousarray(ids, np.uint8)), grank(to), group=group)

    def recv_ids(frm):
        n = torch.zeros(1, dtype=torch.int64)
        dist.recv(n, grank(frm), group=group)
        ids = torch.zeros((int(n.item()), 16), dtype=torch.uint8)
        if int(n.item()):
            dist.recv(ids, grank(frm), group=group)
        return ids.numpy()

    def send_wire(w, to):
        a = np.ascontiguousarray(w, np.uint8) if w is not None else np.zeros(0, np.uint8)
        dist.send(torch.tensor([a.size], dtype=torch.int64), grank(to), group=group)
        if a.size:
            dist.send(torch.from_numpy(a), grank(to), group=group)

    def recv_wire(frm):
        n = torch.zeros(1, dtype=torch.int64)
        dist.recv(n, grank(frm), group=group)
        if not int(n.item()):
            return None
        a = torch.zeros(int(n.item()), dtype=torch.uint8)
        dist.recv(a, grank(frm), group=group)
        return a.numpy()

    # 1. this rank's speculative search (a worker thread, so a drop can cancel it)
    box = {}

    def work():
        try:
            box["wire"] = _wire_of(search(None, query_id))
        except TsgError as e:
            box["err"] = e

    if rank != dst:
        ctrl = torch.full((1,), -1, dtype=torch.int64)
        creq = dist.irecv(ctrl, gdst, group=group)
        th = threading.Thread(target=work, daemon=True)
        th.start()
        # the control message can come while the search runs: a drop cancels it
        got_ctrl = threading.Event()

        def watch():
            creq.wait()
            got_ctrl.set()
            if int(ctrl.item()) == _CTRL_DROP and query_id and th.is_alive():
                cancel(query_id)
        wt = threading.Thread(target=watch, daemon=True)
        wt.start()
        th.join()
        dropped = got_ctrl.is_set() and int(ctrl.item()) == _CTRL_DROP
        if "err" in box and not (box["err"].code == 5 and dropped):  # (TSG_E_CANCELLED after a drop)
            raise box["err"]
        wire = box.get("wire")
        # report: the distinct IDs of this rank's result, in order (empty after a drop)
        send_ids(_distinct_in_order(from_wire(wire)) if wire is not None else np.zeros((0, 16), np.uint8), dst)
        wt.join()
        code = int(ctrl.item())
        if code == _CTRL_SEEDED:
            seen = recv_ids(dst)
            wire = _wire_of(search(seen, 0))
        send_wire(wire if code != _CTRL_DROP else None, dst)
        return None

    # dst: its own search first (its blocks come first when dst = 0), then the reports in order
    work()
    if "err" in box:
        raise box["err"]
    seen_ids, seen_set = [], set()
    stop_at = None
    codes = {}
    for r in range(world):
        ids = _distinct_in_order(from_wire(box["wire"])) if r == dst else recv_ids(r)
        if stop_at is not None:
            continue  # (a rank past the stop: its report is read and dropped)
        before = np.array(seen_ids, np.uint8).reshape(-1, 16)
        reached = False
        for x in ids:
            k = x.tobytes()
            if k not in seen_set:
                seen_set.add(k)
                seen_ids.append(x)
                if limit > 0 and len(seen_set) >= limit:  # (limit <= 0: every match, no stop)
                    reached = True
                    break
        if reached:
            stop_at = r
            codes[r] = (_CTRL_SEEDED if len(before) else _CTRL_KEEP, before)
            for q in range(r + 1, world):
                codes[q] = (_CTRL_DROP, None)
                if q != dst:
                    dist.send(torch.tensor([_CTRL_DROP], dtype=torch.int64), grank(q), group=group)
        else:
            codes[r] = (_CTRL_KEEP, None)
        if r != dst:
            code = codes[r][0]
            if code != _CTRL_DROP:
                dist.send(torch.tensor([code], dtype=torch.int64), grank(r), group=group)
                if code == _CTRL_SEEDED:
                    send_ids(codes[r][1], r)
    # 3. the kept responses, in rank order
    parts = []
    for r in range(world):
        if r == dst:
            code, before = codes[r]
            w = box["wire"] if code == _CTRL_KEEP else (_wire_of(search(before, 0)) if code == _CTRL_SEEDED else None)
        else:
            w = recv_wire(r)
        if w is not None:
            parts.append(from_wire(w))
    return concat_responses(parts)
