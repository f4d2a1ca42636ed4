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
"""
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
