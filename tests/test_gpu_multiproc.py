"""Multi-process engine path on the GPU: one process per rank, each with
its own libtsg context on the device, searching its block shard through the engine
(instance.Search: limit cut, combine, sort), the responses gathered to rank 0 as packed
byte tensors over gloo and merged with the frontend rule
(modules/frontend/searchsharding.go:32-125). The one-GPU box runs both ranks on cuda:0
(RCCL needs a GPU per rank; the 8-GPU form is bench.py's merge leg). Expected: the same
merge applied to the oracle's per-shard querier responses."""
import json
import os
import socket
import tempfile

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
import tempo_amd as T
from tempo_amd import shard

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
QUERY = dict(tags={"service.name": "svc-07", "http.method": "get"}, min_ms=10, max_ms=1000,
             start=T0 + 900, end=T0 + 2700)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _key(res):
    traces, met = res
    return [[[t.trace_id_hex, t.start_time_unix_nano, t.duration_ms, t.root_service_name, t.root_trace_name]
             for t in traces], [met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks]]


def _worker(rank, world, port, paths, limit, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = T.Engine(devices=[0])
    try:
        mine = [eng.open_block(paths[i]) for i in shard.shard_range(len(paths), world, rank)]
        req = T.SearchRequest(tags=QUERY["tags"], min_duration_ms=QUERY["min_ms"], max_duration_ms=QUERY["max_ms"],
                              start=QUERY["start"], end=QUERY["end"], limit=limit)
        res = shard.distributed_search_packed(lambda: eng.search_request(mine, req, limit), limit, len(paths))
        if rank == 0:
            with open(os.path.join(outdir, "merged.json"), "w") as f:
                json.dump(_key(res), f)
        else:
            assert res is None
        for b in mine:
            b.close()
    finally:
        eng.close()
        dist.destroy_process_group()


def _oracle_response(paths, limit):
    got, met, _ = O.search([O.Block(p) for p in paths], limit=limit, combine=limit, **QUERY)
    traces = [T.TraceSearchMetadata(trace_id=m["id"], trace_id_len=m["id_len"],
                                    root_service_name=m["root_service"].decode(),
                                    root_trace_name=m["root_name"].decode(), start_time_unix_nano=m["start_ns"],
                                    duration_ms=m["duration_ms"], end_time_unix_nano=m["end_ns"]) for m in got]
    return traces, T.SearchMetrics(met["traces_inspected"], met["bytes_inspected"], met["blocks_inspected"],
                                   met["blocks_skipped"])


@pytest.mark.parametrize("limit", [20, 5000])
def test_two_rank_engines_gather_and_merge(limit):
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i in range(6):
            p = os.path.join(td, "b%d" % i)
            T.synth_search_block(p, 30_000 + 1_000 * i, seed=500 + i, profile=0, encoding=T.ENC_SNAPPY,
                                 page_size=64 << 10)
            paths.append(p)
        world = 2
        mp.spawn(_worker, args=(world, _free_port(), paths, limit, td), nprocs=world, join=True)
        with open(os.path.join(td, "merged.json")) as f:
            got = json.load(f)
        resp = [_oracle_response([paths[i] for i in shard.shard_range(len(paths), world, r)], limit)
                for r in range(world)]
        exp = _key(shard.merge_responses(resp, limit, len(paths)))
        assert got == exp
        assert len(got[0]) > 0
