"""Rank-sharded search on the GPU: one libtsg context per rank on the
device, each searching its block shard through the engine (instance.Search: limit cut,
combine, sort), each response packed by libtsg into the wire buffer the gather moves
(Engine.search_wire -> tsg_result_pack), merged in libtsg with the frontend rule
(modules/frontend/searchsharding.go:32-125). Expected: the same merge applied to the
oracle's per-shard querier responses. The transport itself (gloo / RCCL gather of the
packed tensors) is covered by test_shard_gloo.py; ranks as processes by bench.py's merge
leg at N > 1. (In-process contexts: this pytest process has initialised the GPU, so it
starts no rank processes.)"""
import os
import tempfile

import pytest

from oracle import oracle as O
import tempo_amd as T
from tempo_amd import shard

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000
QUERY = dict(tags={"service.name": "svc-07", "http.method": "get"}, min_ms=10, max_ms=1000,
             start=T0 + 900, end=T0 + 2700)


def _key(res):
    traces, met = res
    return ([(t.trace_id_hex, t.start_time_unix_nano, t.duration_ms, t.root_service_name, t.root_trace_name)
             for t in traces], (met.inspected_traces, met.inspected_bytes, met.inspected_blocks, met.skipped_blocks))


def _oracle_response(paths, limit):
    got, met, _ = O.search([O.Block(p) for p in paths], limit=limit, combine=limit, **QUERY)
    traces = [T.TraceSearchMetadata(trace_id=m["id"], trace_id_len=m["id_len"],
                                    root_service_name=m["root_service"].decode(),
                                    root_trace_name=m["root_name"].decode(), start_time_unix_nano=m["start_ns"],
                                    duration_ms=m["duration_ms"], end_time_unix_nano=m["end_ns"]) for m in got]
    return traces, T.SearchMetrics(met["traces_inspected"], met["bytes_inspected"], met["blocks_inspected"],
                                   met["blocks_skipped"])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("limit", [20, 5000])
def test_rank_contexts_pack_and_merge(world, limit):
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i in range(6):
            p = os.path.join(td, "b%d" % i)
            T.synth_search_block(p, 30_000 + 1_000 * i, seed=500 + i, profile=0, encoding=T.ENC_SNAPPY,
                                 page_size=64 << 10)
            paths.append(p)
        req = T.SearchRequest(tags=QUERY["tags"], min_duration_ms=QUERY["min_ms"], max_duration_ms=QUERY["max_ms"],
                              start=QUERY["start"], end=QUERY["end"], limit=limit)
        wires = []
        for r in range(world):  # one context per rank, its shard resident on the device
            eng = T.Engine(devices=[0])
            try:
                mine = [eng.open_block(paths[i]) for i in shard.shard_range(len(paths), world, r)]
                # instance.Search's consumer (limit cut, combine, sort), packed: what the gather moves
                wires.append(eng.search_wire(mine, T.Pipeline(req), limit=limit, combine=limit))
                for b in mine:
                    b.close()
            finally:
                eng.close()
        m = shard.merge_wires(wires, limit, len(paths))
        got = _key((m.traces(), m.metrics))
        exp = _key(shard.merge_responses(
            [_oracle_response([paths[i] for i in shard.shard_range(len(paths), world, r)], limit)
             for r in range(world)], limit, len(paths)))
        assert got == exp and len(got[0]) > 0


def test_rccl_gather_world1(engine):
    """The packed gather on cuda tensors through the nccl backend (RCCL) — the transport
    bench.py's merge / cfg5 legs use at N > 1 — in a world of one: the merged response equals
    the host merge of the same wire, and the id-sharded lookup's gathered hit table equals the
    local one."""
    import socket

    import numpy as np
    import torch
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        with tempfile.TemporaryDirectory() as td:
            paths = []
            for i in range(3):
                p = os.path.join(td, "b%d" % i)
                T.synth_search_block(p, 40_000, seed=800 + i, page_size=64 << 10)
                paths.append(p)
            blocks = [engine.open_block(p) for p in paths]
            req = T.SearchRequest(tags=QUERY["tags"], min_duration_ms=QUERY["min_ms"],
                                  max_duration_ms=QUERY["max_ms"], start=QUERY["start"], end=QUERY["end"])
            wire = engine.search_wire(blocks, T.Pipeline(req))
            merged = shard.distributed_search_packed(lambda: wire, 1 << 30, len(paths), device="cuda", columns=True)
            host = shard.merge_wires([wire], 1 << 30, len(paths))
            assert len(merged) == len(host) > 0 and (merged.recs == host.recs).all()
            assert merged.metrics.inspected_traces == host.metrics.inspected_traces
            for b in blocks:
                b.close()
            v2 = []
            for i in range(4):
                p = os.path.join(td, "v%d" % i)
                v2.append((p, T.synth_v2_block(p, 3000, seed=60 + i)))
            vb = [engine.open_v2block(p) for p, _ in v2]
            ids = np.concatenate([x[::7] for _, x in v2] + [np.arange(16 * 500, dtype=np.uint8).reshape(500, 16)])
            local, _ = engine.lookup(vb, ids)
            got = shard.distributed_lookup(lambda x: engine.lookup(vb, x)[0], ids, device="cuda")
            np.testing.assert_array_equal(got, local)
            for b in vb:
                b.close()
    finally:
        dist.destroy_process_group()
