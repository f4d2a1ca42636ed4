"""Multi-GPU search: block sharding over ranks and the frontend's response merge.

One process per GPU. The search path partitions by block (the frontend shards a
query into per-block jobs, modules/frontend/searchsharding.go:325-367), so each
rank searches only its own resident blocks with no data-path collective. The one
exchange is the final, small gather of per-rank responses to rank 0, which then
merges them the way the frontend's `searchResponse` does
(searchsharding.go:32-125):

* `addResponse` (searchsharding.go:71-86): traces keyed by trace ID, first one
  seen wins (no CombineSearchResults here); InspectedBytes / InspectedTraces /
  SkippedBlocks summed; InspectedBlocks is set by the sharder to the number of
  blocks in the query (searchsharding.go:221), not summed.
* `shouldQuit` (searchsharding.go:88-105): stop taking responses once the map
  holds more than `limit` traces.
* `result` (searchsharding.go:107-125): traces sorted by start time descending.

The reference consumes job responses in completion order (racy); here they are
consumed in rank order, and the sort is stable (ties keep first-seen order),
which makes the merged response deterministic.

Two transports for the gather: `distributed_search` pickles the responses
(`gather_object`: fine for limit-bounded responses), `distributed_search_packed`
packs them into two byte tensors (fixed 68-byte records + a names blob) and
gathers those with `dist.gather` — on the GPUs (backend "nccl" = RCCL) the bytes
move device to device over xGMI, which is what a GB-scale full-scan match list
needs. Both merge identically.

Trace-ID lookup shards the probe ids instead (bloom + index replicated on every
rank, tempodb.Find's fan-out over blocks stays rank-local): `shard_ids` gives each
rank a contiguous id slice and `distributed_lookup` gathers the per-rank hit
tables (int64 rows id, block, record, start, length); concatenated in rank order
they are already sorted by (id, block).
"""
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .tsg import SearchMetrics, TraceSearchMetadata


def shard_range(n_blocks: int, world: int, rank: int) -> range:
    """Contiguous block range owned by `rank` (blocks keep their global order)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return range(n_blocks * rank // world, n_blocks * (rank + 1) // world)


@dataclass
class SearchResponse:
    """searchsharding.go:32-125, consumed in a fixed order."""
    limit: int
    inspected_blocks: int = 0
    inspected_bytes: int = 0
    inspected_traces: int = 0
    skipped_blocks: int = 0
    traces: Dict[str, TraceSearchMetadata] = field(default_factory=dict)

    def add_response(self, traces: Sequence[TraceSearchMetadata], metrics: SearchMetrics) -> None:
        for t in traces:
            key = t.trace_id_hex  # the map key is the hex TraceID string
            if key not in self.traces:
                self.traces[key] = t
        self.inspected_bytes += metrics.inspected_bytes
        self.inspected_traces += metrics.inspected_traces
        self.skipped_blocks += metrics.skipped_blocks

    def should_quit(self) -> bool:
        return len(self.traces) > self.limit

    def result(self) -> Tuple[List[TraceSearchMetadata], SearchMetrics]:
        out = sorted(self.traces.values(), key=lambda t: -t.start_time_unix_nano)
        return out, SearchMetrics(self.inspected_traces, self.inspected_bytes, self.inspected_blocks,
                                  self.skipped_blocks)


def merge_responses(responses: Sequence[Tuple[Sequence[TraceSearchMetadata], SearchMetrics]],
                    limit: int, total_blocks: int) -> Tuple[List[TraceSearchMetadata], SearchMetrics]:
    """Frontend merge of per-shard responses, in shard order."""
    r = SearchResponse(limit=limit, inspected_blocks=total_blocks)
    for traces, met in responses:
        if r.should_quit():
            break
        r.add_response(traces, met)
    return r.result()


def distributed_search(search_local: Callable[[], Tuple[List[TraceSearchMetadata], SearchMetrics]],
                       limit: int, total_blocks: int, group=None, dst: int = 0
                       ) -> Optional[Tuple[List[TraceSearchMetadata], SearchMetrics]]:
    """Run this rank's search, gather the responses on `dst`, merge there.

    `search_local` returns this rank's querier response (e.g.
    `Engine.search_request` over the rank's blocks). Returns the merged
    response on `dst`, None elsewhere. Works on any torch.distributed backend
    (gloo for CPU tests, nccl = RCCL on the GPUs)."""
    import torch.distributed as dist
    mine = search_local()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    got = [None] * world if rank == dst else None
    dist.gather_object(mine, got, dst=dst, group=group)
    if rank != dst:
        return None
    return merge_responses(got, limit, total_blocks)


# ---- packed transport (tensors, not pickles) -------------------------------------
# record: id[16] | id_len u8 | pad[3] | duration_ms u32 | start_ns u64 | end_ns u64 |
#         entry_idx u64 | block_idx u32 | service off u32, len u32 | name off u32, len u32
_REC = struct.Struct("<16sB3xIQQQIIIII")
assert _REC.size == 68


def pack_traces(traces: Sequence[TraceSearchMetadata]):
    """(records bytes, names bytes) for a response's traces, in order."""
    recs = bytearray()
    names = bytearray()
    for t in traces:
        svc = t.root_service_name.encode()
        nm = t.root_trace_name.encode()
        so, no = len(names), len(names) + len(svc)
        names += svc + nm
        recs += _REC.pack(bytes(t.trace_id).ljust(16, b"\0")[:16], t.trace_id_len, t.duration_ms,
                          t.start_time_unix_nano, t.end_time_unix_nano, t.entry_idx, t.block_idx,
                          so, len(svc), no, len(nm))
    return bytes(recs), bytes(names)


def unpack_traces(recs: bytes, names: bytes) -> List[TraceSearchMetadata]:
    out = []
    for i in range(len(recs) // _REC.size):
        (tid, tlen, dur, st, en, ent, blk, so, sl, no, nl) = _REC.unpack_from(recs, i * _REC.size)
        out.append(TraceSearchMetadata(trace_id=tid, trace_id_len=tlen,
                                       root_service_name=names[so:so + sl].decode(),
                                       root_trace_name=names[no:no + nl].decode(), start_time_unix_nano=st,
                                       duration_ms=dur, end_time_unix_nano=en, block_idx=blk, entry_idx=ent))
    return out


def _gather_bytes(parts: Sequence[bytes], device, group, dst):
    """Gather variable-length byte strings (one list per rank) to `dst` as tensors:
    sizes first (one int64 per part), then every part padded to the longest."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = torch.tensor([len(p) for p in parts], dtype=torch.int64, device=device)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)] if rank == dst else None
    dist.gather(sizes, all_sizes, dst=dst, group=group)
    # the longest part of any rank: a max all-reduce, so every rank pads alike
    mx = sizes.max().clone() if len(parts) else torch.zeros((), dtype=torch.int64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    width = max(1, int(mx.item()))
    buf = torch.zeros((len(parts), width), dtype=torch.uint8, device=device)
    for i, p in enumerate(parts):
        if p:
            buf[i, :len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8).to(device)
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    out = []
    for r in range(world):
        sz = all_sizes[r].cpu().tolist()
        host = bufs[r].cpu().numpy()
        out.append([host[i, :sz[i]].tobytes() for i in range(len(parts))])
    return out


def distributed_search_packed(search_local: Callable[[], Tuple[List[TraceSearchMetadata], SearchMetrics]],
                              limit: int, total_blocks: int, device=None, group=None, dst: int = 0
                              ) -> Optional[Tuple[List[TraceSearchMetadata], SearchMetrics]]:
    """`distributed_search` with the responses moved as byte tensors on `device`
    (a CUDA device with the nccl backend: RCCL over xGMI; the CPU with gloo)."""
    import torch.distributed as dist
    traces, met = search_local()
    recs, names = pack_traces(traces)
    mets = struct.pack("<QQQQ", met.inspected_traces, met.inspected_bytes, met.inspected_blocks,
                       met.skipped_blocks)
    got = _gather_bytes([recs, names, mets], device or "cpu", group, dst)
    if dist.get_rank(group) != dst:
        return None
    responses = []
    for r_recs, r_names, r_mets in got:
        it, ib, ibl, sk = struct.unpack("<QQQQ", r_mets)
        responses.append((unpack_traces(r_recs, r_names), SearchMetrics(it, ib, ibl, sk)))
    return merge_responses(responses, limit, total_blocks)


def shard_ids(n_ids: int, world: int, rank: int) -> range:
    """Contiguous probe-id slice owned by `rank` (config 5: 10 M ids over the GPUs)."""
    return shard_range(n_ids, world, rank)


def distributed_lookup(lookup_local: Callable[[object], object], ids, device=None, group=None, dst: int = 0):
    """Each rank looks up its id slice against every (replicated) block; rank `dst`
    returns the global hit table (int64 rows: id, block, record, start, length) sorted
    by (id, block), others None. `lookup_local(id_slice)` returns the rank's table with
    slice-local id indices (e.g. `lambda x: engine.lookup(blocks, x)[0]`)."""
    import numpy as np
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sl = shard_ids(len(ids), world, rank)
    hits = np.asarray(lookup_local(ids[sl.start:sl.stop]), dtype=np.int64).reshape(-1, 5).copy()
    hits[:, 0] += sl.start
    got = _gather_bytes([hits.tobytes()], device or "cpu", group, dst)
    if rank != dst:
        return None
    return np.concatenate([np.frombuffer(g[0], dtype=np.int64).reshape(-1, 5) for g in got])
