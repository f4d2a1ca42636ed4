#!/usr/bin/env python3
"""BASELINE config 5: batched trace-ID lookup (bloom + index) over v2 blocks.

Not the bench.py headline line (that is config 2); prints one JSON line with
probes/s for the lookup path. Probes: half are ids present in some block, half
random (absent); every probe is tested against every resident block, as
tempodb.Find's per-block FindTraceByID fan-out would (tempodb/tempodb.go:288-364).
Checked against the oracle on a sample of probes.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=200)
    ap.add_argument("--objects", type=int, default=100_000, help="trace objects per block")
    ap.add_argument("--probes", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--check", type=int, default=2000, help="probes checked against the oracle")
    args = ap.parse_args()
    import numpy as np
    import tempo_amd as T

    work = tempfile.mkdtemp(prefix="tsg_lookup_", dir="/tmp")
    try:
        t0 = time.time()
        present = []
        paths = []
        for b in range(args.blocks):
            p = os.path.join(work, f"v2_{b}")
            present.append(T.synth_v2_block(p, args.objects, seed=b))
            paths.append(p)
        present = np.concatenate(present)
        gen_s = time.time() - t0
        rng = np.random.default_rng(5)
        half = args.probes // 2
        probes = np.concatenate([present[rng.integers(0, len(present), half)],
                                 rng.integers(0, 256, (args.probes - half, 16), dtype=np.uint8)])
        probes = probes[rng.permutation(len(probes))]
        eng = T.Engine(devices=[0])
        t0 = time.time()
        blocks = [eng.open_v2block(p) for p in paths]
        load_s = time.time() - t0
        hits, _ = eng.lookup(blocks, probes)  # warmup
        times, kns = [], []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            hits, kernel_ns = eng.lookup(blocks, probes)
            times.append(time.perf_counter() - t0)
            kns.append(kernel_ns)
        step = sum(times) / len(times)
        kern = sum(kns) / len(kns) / 1e9
        # oracle spot check on a probe sample
        from oracle import oracle as O
        ob = [O.V2Block(p) for p in paths]
        sample = probes[: args.check]
        rc, exp = O.lookup(ob, sample, nthreads=8)
        got = sorted((int(h[0]), int(h[1]), int(h[2])) for h in hits if h[0] < args.check)
        parity = rc == 0 and got == sorted((int(e[0]), int(e[1]), int(e[2])) for e in exp)
        out = {
            "metric": "trace-ID lookups/sec (config 5 shape)", "value": args.probes / step, "unit": "probes/s",
            "probe_block_pairs_per_s": args.probes * args.blocks / step, "kernel_s": kern, "step_s": step,
            "blocks": args.blocks, "objects_per_block": args.objects, "probes": args.probes,
            "hits": int(len(hits)), "parity_sample": parity, "gen_s": gen_s, "load_s": load_s,
        }
        print(json.dumps(out), flush=True)
        for b in blocks:
            b.close()
        eng.close()
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
