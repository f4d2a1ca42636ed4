#!/usr/bin/env python3
"""Benchmark: Tempo backend search on MI355X (BASELINE.json configs[1], "config 2").

One step = one full search (tsg_search) of a resident 10 M-entry block set with the
config-2 query: {service.name: svc-07, http.method: get, status.code: error}
+ MinDurationMs=10 + MaxDurationMs=1000 + Start/End over the middle 50 % of
the one-hour window, limit 0 (every match, ordered). Inputs are resident in HBM
before the timed region; each step includes the dictionary match, the scan +
compaction kernel, the records landing in pinned host memory and host result
assembly (names resolved), i.e. what the Go shim receives.

HBM regime: the set is resident --sets (4) times as disjoint copies (tsg_block_clone)
and step i searches copy i % 4, so 4 x 150 MB of filter columns rotate through the
256 MiB Infinity Cache and every step streams from HBM (roofline.regime "hbm").
The same-copy-every-step number (round 1's, MALL-resident) is reported as "mall".

Multi-GPU: one process per GPU. `--gpus N` under torchrun (WORLD_SIZE set) runs as
one rank; `--gpus N` without it starts the N ranks itself (torch.distributed.run as a
child process, before anything touches a GPU) and exits with their status, failing
if fewer than N devices are visible. Blocks are sharded by block, each rank holds its
own 10 M entries (weak scaling). Rank timings are bracketed by a barrier + device
sync and the max over ranks is reported. No data-path collective in the main line:
the ranks' ordered match lists are independent per block (the `merge` leg gathers
them the way the frontend does, over gloo and over RCCL).

Legs beside the main line: mall, limit20, shim (limit 0 and 20), concurrent, cfg3
(config 3's per-GPU share: limit-20 early exit vs full scan), cfg4 (config 4 at 10 M
entries), cfg5 (config 5: 10 M probes x 200 v2 blocks, ids sharded over the ranks),
merge (N > 1). Every leg that searches is checked against the oracle after the timed
legs (`parity`), on the host, untimed.

Prints ONE JSON line (rank 0).
"""
import argparse
import gc
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "search entries scanned/sec + achieved HBM GB/s at 1/2/4/8 MI355X"
T0 = 1_700_000_000
QUERY = dict(tags={"service.name": "svc-07", "http.method": "get", "status.code": "error"},
             min_duration_ms=10, max_duration_ms=1000, start=T0 + 900, end=T0 + 2700)
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
T_PATH_RESIDENT = 1  # tsg_metrics.path: served by the resident kernel (tempo_amd.PATH_RESIDENT)
# device of the small timing / count tensors reduced over the ranks: cuda over RCCL, or the
# host under --ranks-share-gpu (several ranks on one GPU: the process group is gloo)
RED_DEVICE = "cuda"
SHARED_GPU = False
# The config-2 query (3 u8 term columns, duration + range filters, 10 blocks) runs
# the one-launch path; TSG_NO_FAST=1 forces the general path (prep + search kernels).
# The last template argument of the one-launch kernel is segment mode (per-workgroup
# record segments; TSG_NO_SEG=1 forces look-back mode).
# Narrow full scans (limit 0) run the pool kernel (one workgroup per CU, CU-wide work
# pool); TSG_NO_POOL=1 keeps them on the one-launch segment kernel.
if os.environ.get("TSG_NO_FAST"):
    KERNEL = "search_kernel<3, true, true, true>"
elif os.environ.get("TSG_NO_SEG"):
    KERNEL = "search_fast_kernel<3, true, true, true, false>"
elif os.environ.get("TSG_NO_POOL") or os.environ.get("TSG_NO_NARROW"):
    KERNEL = "search_fast_kernel<3, true, true, true, true>"
else:
    KERNEL = "search_pool_kernel<3, true, true, %s>" % ("false" if os.environ.get("TSG_POOL_NT", "1") == "0" else "true")
# HBM-side bytes per launch of KERNEL from separate rocprofv3 --pmc passes
# (FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE), written by
# tools/pmc_summary.py --out; keyed by workload so other sizes report null.
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(workload_key, kernel=None):
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    w = d.get(workload_key, {})
    for name, ent in w.items():
        if (kernel or KERNEL).replace(" ", "") in name.replace(" ", ""):  # rocprof: "void tsg::search_fast_kernel<...>(tsg::QArgs)"
            return ent.get("traffic_bytes_per_launch"), ent.get("source", w.get("_source"))
    return None, None


def summary(out):
    """The headline figures of every leg in a few keys, emitted as the line's last key (the
    driver keeps the tail of long output: these stay visible there)."""
    def g(*path):
        d = out
        for k in path:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return round(d, 3) if isinstance(d, float) else d
    s = {"value_G": round(out["value"] / 1e9, 2) if out.get("value") else None,
         "frac": g("roofline", "frac"), "kernel_avg_us": g("roofline", "avg_launch_us"),
         "step_us_mean": g("latency_us", "step", "mean"), "step_us_p50": g("latency_us", "step", "p50"),
         "mall_frac": g("mall", "frac"), "limit20_step_us_mean": g("limit20", "step_us", "mean"),
         "limit20_kernel_us_p50": g("limit20", "kernel_us", "p50"),
         "shim_query_us_p50": g("shim", "query_us", "p50"), "shim_limit20_us_p50": g("shim", "limit20", "query_us", "p50"),
         "shim_limit20_us_p99": g("shim", "limit20", "query_us", "p99"),
         "cfg3_kernel_us_p50": g("cfg3", "full_scan", "kernel_us", "p50"), "cfg3_frac": g("cfg3", "full_scan", "frac"),
         "cfg3_first20_us_p50": g("cfg3", "limit20", "time_to_first_20_us", "p50"),
         "cfg5_device_ms": g("cfg5", "device_ms"), "cfg5_host_e2e_ms_p50": g("cfg5", "host_e2e", "step_ms", "p50"),
         "load_gb_per_s": g("load_gb_per_s"), "cfg4_load_gb_per_s": g("cfg4", "load_gb_per_s"),
         "cfg1_kernel_us_p50": g("cfg1", "gpu", "kernel_us", "p50"),
         "batched_device_us_per_query": g("batched", "device_us_per_query"), "batched_frac": g("batched", "frac"),
         "batched_wall_us_per_query": g("batched", "wall_us_per_query"),
         "merged_shm_step_us_p50": g("merge", "shm", "step_us", "p50"), "merged_gloo_step_us_p50": g("merge", "step_us", "p50")}
    for name, q in (g("cfg4", "queries") or {}).items():
        s["cfg4_" + name] = {"step_over_device": round(q["step_over_device"], 3) if q.get("step_over_device") else None,
                             "scan_us_p50": round(q["scan_us"]["p50"], 1), "dict_frac": round(q["dict_frac"], 3)
                             if q.get("dict_frac") else None}
    s["parity"] = {k: g(k, "parity", "ok") for k in ("cfg1", "cfg3", "cfg4", "cfg5") if k in out}
    s["cpu_baseline_entries_per_s"] = g("cpu_baseline", "value")
    return s


def pct(xs):
    """p10 / median / p90 of a sample (SURVEY.md §8(d) timing rules)."""
    if not xs:
        return None
    v = sorted(xs)
    at = lambda q: v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]  # noqa: E731
    return {"p10": at(0.1), "p50": at(0.5), "p90": at(0.9), "p99": at(0.99), "mean": sum(v) / len(v), "max": v[-1]}


def node_cpus(node):
    """CPUs of a NUMA node (sysfs cpulist)."""
    try:
        lst = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return set()
    out = set()
    for part in lst.split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def idlest(cpus, k, window=0.3):
    """k CPUs of `cpus` on the k cores with the most idle time over `window` seconds (/proc/stat):
    the GPU box shares its host with other jobs, and a search thread that lands on a
    busy core loses tens of microseconds per step to preemption."""
    def snap():
        out = {}
        try:
            for line in open("/proc/stat"):
                if line.startswith("cpu") and line[3:4].isdigit():
                    f = line.split()
                    out[int(f[0][3:])] = int(f[4]) + int(f[5])  # idle + iowait
        except OSError:
            pass
        return out
    a = snap()
    time.sleep(window)
    b = snap()
    idle = {c: b.get(c, 0) - a.get(c, 0) for c in cpus}
    # whole cores: a CPU whose SMT sibling is busy shares its core's issue slots, so a
    # core counts as idle as its busiest thread; one CPU per core, the k idlest cores
    cores = {}
    for c in cpus:
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        cores.setdefault(sib, []).append(c)
    ranked = sorted(cores.values(), key=lambda th: (-min(idle[t] for t in th), min(th)))
    pick = [min(th) for th in ranked[:k]]
    if len(pick) < k:  # (fewer cores than k: fill with the idlest remaining CPUs)
        rest = sorted((c for c in cpus if c not in pick), key=lambda c: -idle[c])
        pick += rest[:k - len(pick)]
    return sorted(pick)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=10, help="blocks per GPU (one config-2 set)")
    ap.add_argument("--entries", type=int, default=1_000_000, help="entries per block")
    ap.add_argument("--sets", type=int, default=4,
                    help="disjoint resident copies of the block set (tsg_block_clone), searched in rotation: "
                         "4 x 150 MB of filter columns >> the 256 MiB Infinity Cache, so every step streams "
                         "from HBM (roofline.regime 'hbm'); 1 = the same set every step ('mall')")
    ap.add_argument("--mall-steps", type=int, default=100,
                    help="extra timed steps on one set (the MALL-resident regime), reported beside; 0 = skip")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on the host (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baselines (0 = this job's CPU share: the process's CPUs, at most 16, "
                         "the GPU box's per-GPU share)")
    ap.add_argument("--events", type=int, default=4,
                    help="HIP events around the search kernel of every N-th timed step (roofline.achieved: "
                         "the average over those launches); 0 = off")
    ap.add_argument("--batch-queries", type=int, default=64,
                    help="batched leg: config-2 queries per tsg_search_batch call (SURVEY §8(d) batched mode; 0 = skip)")
    ap.add_argument("--batch-depth", type=int, default=8, help="batched leg: searches in flight at once")
    ap.add_argument("--batch-reps", type=int, default=6, help="batched leg: timed batches")
    ap.add_argument("--limit-steps", type=int, default=20,
                    help="extra timed searches with limit=20 (early exit, config-3 mode); 0 = skip")
    ap.add_argument("--cfg3", type=int, default=None,
                    help="config-3 leg on this GPU's share: --cfg3-blocks resident blocks of --cfg3-entries "
                         "(one generated block + device clones), full scan x --cfg3-steps back-to-back queries "
                         "and limit=20 (time to the first 20); 0 = skip (default: on at N=1 only — the "
                         "multi-GPU runs keep to the config-2 line and its disk/HBM footprint)")
    ap.add_argument("--streams", type=int, default=4,
                    help="concurrent leg: query streams (device contexts on this GPU, each with its own HIP "
                         "stream, pinned output and resident copy of the set) driven by as many host threads")
    ap.add_argument("--concurrent-steps", type=int, default=64,
                    help="queries per stream in the concurrent leg (0 = skip)")
    ap.add_argument("--shim-steps", type=int, default=200,
                    help="queries in the shim-pattern leg (one C thread per block, a tsg_search each; 0 = off)")
    ap.add_argument("--merge-steps", type=int, default=20,
                    help="N > 1: distributed full-scan queries with the frontend merge on rank 0 (0 = off)")
    ap.add_argument("--cfg4", type=int, default=None, help="config-4 leg (default: on at N=1)")
    ap.add_argument("--cfg4-blocks", type=int, default=10,
                    help="config-4 blocks: one generated block of --cfg4-entries + device clones")
    ap.add_argument("--cfg4-entries", type=int, default=1_000_000)
    ap.add_argument("--cfg4-steps", type=int, default=10)
    ap.add_argument("--cfg3-blocks", type=int, default=25)
    ap.add_argument("--cfg3-entries", type=int, default=5_000_000)
    ap.add_argument("--cfg3-steps", type=int, default=64)
    ap.add_argument("--cfg1", type=int, default=1,
                    help="config-1 leg (rank 0): one 1 M-entry block, one tag=value; GPU steps + the CPU pipeline "
                         "restated (single thread and the reference harness's 10-thread shape) after the GPU legs")
    ap.add_argument("--cfg1-steps", type=int, default=100)
    ap.add_argument("--cfg5", type=int, default=1, help="config-5 leg: batched trace-ID lookup (0 = skip)")
    ap.add_argument("--cfg5-blocks", type=int, default=200)
    ap.add_argument("--cfg5-objects", type=int, default=100_000)
    ap.add_argument("--cfg5-probes", type=int, default=10_000_000, help="probes over all ranks (sharded by id)")
    ap.add_argument("--cfg5-steps", type=int, default=5)
    ap.add_argument("--parity", type=int, default=1, help="oracle parity of the cfg3/cfg4/cfg5 legs (untimed)")
    ap.add_argument("--ranks-share-gpu", action="store_true",
                    help="N > 1 on fewer GPUs: every rank on device 0 with a gloo process group (a rehearsal "
                         "of the multi-rank legs on a 1-GPU lease; RCCL legs are reported as skipped)")
    ap.add_argument("--pin", default="auto", choices=["auto", "none"],
                    help="auto: keep this process on the CPUs of its GPU's NUMA node (tsg_device_numa_node)")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--keep", action="store_true")
    return ap.parse_args()


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(argv, n, port):
    """The torch.distributed.run command that starts `n` ranks of this script (one per GPU,
    rendezvous on 127.0.0.1) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def rank_env(args, env=None):
    """(rank, world, local rank) of this process, or None when `--gpus N` asks this process
    to start the ranks itself (N > 1 and no torchrun environment). A torchrun world that
    differs from --gpus is an error."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if args.gpus not in (1, world):  # (--gpus 1 under an outer torchrun: the world decides)
            raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
        return int(env.get("RANK", "0")), world, int(env.get("LOCAL_RANK", "0"))
    if args.gpus <= 1:
        return 0, 1, 0
    return None


def launch_ranks(args, argv, device_count=None):
    """`--gpus N` without torchrun: start N ranks as a child process group and return
    their exit status. Runs before anything touches a GPU (no HIP call in this process:
    torch.cuda.device_count() does not initialise the device on this image)."""
    if device_count is None:
        import torch
        device_count = torch.cuda.device_count()
    if device_count < args.gpus and not (args.ranks_share_gpu and device_count >= 1):
        print(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {device_count}",
              file=sys.stderr, flush=True)
        return 2
    cmd = launch_cmd(argv, args.gpus, free_port())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.ranks_share_gpu:
        # ranks sharing one GPU: no resident search kernels (each would hold every CU's LDS and
        # the other rank's queries would wait for it to leave on its idle timeout)
        env.setdefault("TSG_RESIDENT", "0")
    log("starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd, env=env)


def columns_vs_oracle(cols, gmet, exp, omet, nrep):
    """GPU result (Engine.search_columns) over `nrep` byte-identical device copies of one block
    vs the oracle's result on that block: copy r must hold exactly the oracle's matches, in
    order, with block index r, every field equal (id, scan position, start, end, DurationMs,
    root names); the metrics are nrep times the oracle's."""
    import numpy as np
    keys = ("traces_inspected", "bytes_inspected", "blocks_inspected", "blocks_skipped")
    got_m = (gmet.inspected_traces, gmet.inspected_bytes, gmet.inspected_blocks, gmet.skipped_blocks)
    if got_m != tuple(nrep * omet[k] for k in keys):
        return False
    n1 = len(exp)
    if len(cols["start_ns"]) != n1 * nrep:
        return False
    if n1 == 0:
        return True
    eid = np.frombuffer(b"".join(m["id"] for m in exp), np.uint8).reshape(n1, 16)
    col = lambda f, dt: np.fromiter((m[f] for m in exp), dt, n1)  # noqa: E731
    e_entry, e_start, e_end = col("entry_idx", np.uint64), col("start_ns", np.uint64), col("end_ns", np.uint64)
    e_dur = col("duration_ms", np.uint32)
    nidx = {s: i for i, s in enumerate(cols["names"])}
    e_svc = np.fromiter((nidx.get(m["root_service"], -1) for m in exp), np.int64, n1)
    e_nm = np.fromiter((nidx.get(m["root_name"], -1) for m in exp), np.int64, n1)
    for r in range(nrep):
        s = slice(r * n1, (r + 1) * n1)
        if not ((cols["block_idx"][s] == r).all() and (cols["entry_idx"][s] == e_entry).all()
                and (cols["trace_id"][s] == eid).all() and (cols["start_ns"][s] == e_start).all()
                and (cols["end_ns"][s] == e_end).all() and (cols["duration_ms"][s] == e_dur).all()
                and (cols["root_service"][s] == e_svc).all() and (cols["root_name"][s] == e_nm).all()):
            return False
    return True


def oracle_query(q):
    """A bench query (SearchRequest fields) as oracle.search keyword arguments."""
    return dict(tags=q.get("tags", {}), min_ms=q.get("min_duration_ms", 0), max_ms=q.get("max_duration_ms", 0),
                start=q.get("start", 0), end=q.get("end", 0))


def run_parity(jobs):
    """Run the legs' oracle checks (name -> callable) concurrently on the host (the oracle's
    C calls release the GIL); returns name -> result (or the error)."""
    res = {}

    def one(item):
        name, fn = item
        t0 = time.time()
        try:
            r = fn()
        except Exception as e:  # noqa: BLE001  (reported, not raised: the timed figures stand)
            r = {"ok": False, "error": repr(e)}
        r["oracle_s"] = time.time() - t0
        res[name] = r

    parallel(one, list(jobs.items()))
    return res


def gen_blocks(workdir, rank, nblocks, n, threads):
    import tempo_amd as T
    paths = [os.path.join(workdir, f"r{rank}b{i}") for i in range(nblocks)]
    errs = []
    # (a --workdir kept from an earlier run is reused: its blocks are seeded the same)
    todo = [(i, p) for i, p in enumerate(paths) if not os.path.exists(os.path.join(p, "search.meta.json"))]
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                if not todo:
                    return
                i, p = todo.pop(0)
            try:
                T.synth_search_block(p, n, seed=rank * 1000 + i, profile=0, encoding=T.ENC_SNAPPY,
                                     page_size=1024 * 1024)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

    ths = [threading.Thread(target=work) for _ in range(max(1, threads))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    return paths


def parallel(fn, items):
    out = [None] * len(items)
    errs = []

    def run(i):
        try:
            out[i] = fn(items[i])
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(items))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    return out


def batch_leg(args, eng, sets, pipe, entries, scan_bytes, nmatch):
    """SURVEY §8(d)'s batched mode: --batch-queries config-2 queries (the 4 resident copies in
    turn) in one tsg_search_batch call, --batch-depth in flight: the resident kernel takes the next
    query from its mailbox while earlier ones finish, the host assembles earlier results meanwhile.
    device_us_per_query = the batch's resident launch's dispatch duration (AQL dispatch timestamps:
    the clock rocprofv3's kernel trace reads; launch and quit included) / queries."""
    k = args.batch_queries
    items = [(sets[i % len(sets)], pipe) for i in range(k)]
    eng.search_batch(items[: min(k, 16)], depth=args.batch_depth, unpack=False)  # (warm)
    walls, devs, ok = [], [], True
    for _ in range(max(1, args.batch_reps)):
        t0 = time.perf_counter()
        res, dns = eng.search_batch(items, depth=args.batch_depth, unpack=False)
        walls.append(time.perf_counter() - t0)
        devs.append(dns)
        ok = ok and all(n == nmatch for n, _ in res) and all(m.path == T_PATH_RESIDENT for _, m in res)
    wall = sorted(walls)[len(walls) // 2]
    dv = [d for d in devs if d]
    dev = sorted(dv)[len(dv) // 2] if dv else 0
    per_q = dev / k if dev else None
    ach = scan_bytes / per_q if per_q else None  # bytes / ns = GB/s
    return {"queries": k, "depth": args.batch_depth, "reps": len(walls),
            "wall_us_per_query": wall / k * 1e6, "entries_per_s": entries * k / wall,
            "device_us_per_query": per_q / 1e3 if per_q else None,
            "device_us_per_query_all": [round(d / k / 1e3, 3) for d in devs],
            "achieved_gbps": ach, "frac": ach / PEAK_HBM_GBPS if ach else None,
            "bytes_per_query": scan_bytes, "counts_match_and_resident": ok,
            "note": "one resident launch per batch serves every query (its dispatch is what a kernel trace shows); "
                    "device time per query = dispatch duration / queries"}


def cpu_baselines(paths, got, threads, oracle_threads=None):
    """The reference's scan restated (oracle: snappy decode + flatbuffer walk + ContainsTag,
    one thread per block like instance.searchLocalBlocks) and the CPU columnar variant
    (the same predicates over host-decoded columns, `threads` threads), both on this rank's
    set. The oracle leg runs one thread per block over `oracle_threads` block searches (the
    set's blocks cycled: every thread a whole-block search, BASELINE.md row 2's model on as
    many cores as the job may use); parity is checked on one pass over the set. Returns the
    cpu_baseline object."""
    from oracle import oracle as O
    q = dict(tags=QUERY["tags"], min_ms=QUERY["min_duration_ms"], max_ms=QUERY["max_duration_ms"],
             start=QUERY["start"], end=QUERY["end"])
    oblocks = [O.Block(p) for p in paths]
    nb = len(oblocks)
    exp, omet, st = O.search(oblocks, nthreads=nb, **q)
    per_block = omet["traces_inspected"] / nb
    nthr = max(nb, int(oracle_threads or nb))
    work = [oblocks[i % nb] for i in range(nthr)]  # one block search per thread
    t0 = time.perf_counter()
    reps = 0
    while True:
        _, wmet, wst = O.search(work, nthreads=nthr, **q)
        reps += 1
        if time.perf_counter() - t0 > 10 or reps >= 5:
            break
    cpu_s = (time.perf_counter() - t0) / reps
    entries = wmet["traces_inspected"]
    # parity of the GPU's full result against it: every field of every match, in order
    gk = [(m.block_idx, m.entry_idx, m.trace_id, m.start_time_unix_nano, m.end_time_unix_nano, m.duration_ms,
           m.root_service_name.encode(), m.root_trace_name.encode()) for m in got]
    ek = [(m["block_idx"], m["entry_idx"], m["id"], m["start_ns"], m["end_ns"], m["duration_ms"], m["root_service"],
           m["root_name"]) for m in exp]
    out = {
        "value": entries / cpu_s, "unit": "entries/s", "cores": nthr, "kind": "port",
        "sample": f"oracle BackendSearchBlock.Search restatement (snappy decode + flatbuffer walk + ContainsTag "
                  f"included), one thread per block search: {nthr} whole-block searches of 1 M entries at once "
                  f"({nb} distinct blocks of the GPU's set, cycled; {entries} entries), {reps} rep(s); "
                  f"{nthr} threads = this job's CPU share of the box (nproc {os.cpu_count()})",
        "per_thread_entries_per_s": entries / cpu_s / nthr,
        "decompression_included": True,
        "nproc": os.cpu_count(), "cpu_share": len(os.sched_getaffinity(0)), "cpu_model": cpu_model(),
        "parity": st == 0 and wst == 0 and gk == ek and omet["blocks_inspected"] == nb,
        "entries_per_block": per_block,
    }
    # columnar: decode once (not timed, like the GPU's resident columns), then time the scan
    t0 = time.perf_counter()
    cols = parallel(O.ColumnarBlock, oblocks)
    build_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    reps = 0
    while True:
        cm, ch = O.columnar_search(cols, nthreads=threads, **q)
        reps += 1
        if time.perf_counter() - t0 > 5 or reps >= 50:
            break
    col_s = (time.perf_counter() - t0) / reps
    out["columnar"] = {
        "value": omet["traces_inspected"] / col_s, "unit": "entries/s", "cores": threads,
        "sample": f"the same {omet['traces_inspected']} entries decoded once into host columns ({build_s:.1f}s, "
                  f"untimed), Pipeline predicates over the columns on {threads} threads, {reps} rep(s); threads = "
                  f"this job's CPU share of the shared GPU box (of {os.cpu_count()} CPUs there); --cpu-threads overrides",
        "parity": cm == len(got) and ch == O.match_hash([(m.block_idx, m.entry_idx) for m in got]),
    }
    return out


CFG1_QUERY = dict(tags={"service.name": "svc-07"})


def cfg1_leg(args, eng, block, path, steps):
    """BASELINE config 1: one synthetic local-disk search block (1 M traces, ~20 tags each),
    one tag=value matcher. The GPU leg here (tsg_search over that one resident block, timed
    steps); the CPU legs (the reference pipeline restated, the reference harness's shape) run
    after the GPU legs, in the returned closure, with parity of the GPU's matches."""
    import tempo_amd as T
    pipe = T.Pipeline(T.SearchRequest(**CFG1_QUERY))
    blk = (block,)
    cols, gmet = eng.search_columns(list(blk), pipe)
    for _ in range(5):
        eng.search_raw(blk, pipe)
    eng.kernel_times()
    ts = []
    for i in range(steps):
        t0 = time.perf_counter()
        eng.search_raw(blk, pipe, flags=T.SEARCH_TIME_DEFER if i % 4 == 2 else 0, metrics=False)
        ts.append(time.perf_counter() - t0)
    kns = eng.kernel_times()
    entries = gmet.inspected_traces
    res = {"workload": "config 1: one 1 M-entry block (~20 tags per entry, snappy 1 MiB pages), tag=value "
                       "{service.name: svc-07}, full scan", "entries": entries, "matches": len(cols["start_ns"]),
           "gpu": {"steps": steps, "step_us": pct([x * 1e6 for x in ts]), "kernel_us": pct([x / 1e3 for x in kns]),
                   "entries_per_s": entries * steps / sum(ts),
                   "scan_bytes": gmet.scan_bytes}}

    def cpu():
        from oracle import oracle as O
        ob = O.Block(path)
        q = oracle_query(CFG1_QUERY)
        t0 = time.perf_counter()
        exp, omet, st = O.search([ob], **q)
        one_s = time.perf_counter() - t0
        ok = st == 0 and columns_vs_oracle(cols, gmet, exp, omet, 1)
        # the reference harness's shape (backend_search_block_test.go:128-172): 10 goroutines,
        # each searching the block 10 times; here 10 threads x 2 searches (bounded sample)
        loops = 2
        t0 = time.perf_counter()
        for _ in range(loops):
            _, hm, _ = O.search([ob] * 10, nthreads=10, **q)
        h_s = time.perf_counter() - t0
        return {"ok": bool(ok), "checked": "every match (every field, in order) + metrics vs the oracle",
                "cpu_single_thread": {"value": omet["traces_inspected"] / one_s, "unit": "entries/s", "cores": 1,
                                      "kind": "port", "mib_per_s": omet["bytes_inspected"] / one_s / 2**20,
                                      "sample": "one BackendSearchBlock.Search of the block (oracle restatement, "
                                                "snappy decode + flatbuffer walk included)"},
                "cpu_harness_shape": {"value": 10 * loops * omet["traces_inspected"] / h_s, "unit": "entries/s",
                                      "cores": 10, "kind": "port",
                                      "mib_per_s": 10 * loops * omet["bytes_inspected"] / h_s / 2**20,
                                      "sample": f"10 threads x {loops} searches of the block at once (the reference "
                                                f"benchmark runs 10 goroutines x 10)"}}
    return res, cpu


def concurrent_leg(args, base, pipe, streams, entries, dist, world, local):
    """Serving throughput: `streams` query streams on this GPU, each a device context of
    its own (HIP stream, pinned result buffers) searching its own resident copy of the
    config-2 set, one host thread each, --concurrent-steps full-scan queries per stream.
    One query's host work (plan, launch, result assembly) overlaps other streams'
    kernels, so the rate approaches the kernel's; the per-query work is the same as the
    main line's (SURVEY.md 8(d) batched mode: back-to-back queries)."""
    import torch
    import tempo_amd as T
    # (its own engine, created after the main legs: they run with one device context)
    eng = T.Engine(devices=[local] * streams)
    csets = [tuple(b.clone(eng, device=i) for b in base) for i in range(streams)]
    for i, cs in enumerate(csets):  # warm every stream (plans, pinned buffers)
        for _ in range(3):
            eng.search_raw(cs, pipe)
    errs = []
    n = args.concurrent_steps
    go = threading.Barrier(streams + 1)

    def worker(i):
        try:
            go.wait()
            for _ in range(n):
                eng.search_raw(csets[i], pipe, metrics=False)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(streams)]
    for t in ths:
        t.start()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    go.wait()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if errs:
        raise errs[0]
    if dist:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    for cs in csets:
        for b in cs:
            b.close()
    eng.close()
    return {"streams": streams, "queries_per_stream": n,
            "entries_per_s": entries * n * streams * world / elapsed,
            "queries_per_s": n * streams * world / elapsed,
            "note": "one resident copy of the config-2 set per stream; full scans, same query as the main line"}


def shim_leg(args, eng, sets, pipe, entries, nmatch, batched, dist, all_cpus):
    """The Go shim's call pattern for the ingester: searchLocalBlocks starts a goroutine
    per block and each calls Search on its own (instance_search.go:164-185), so the shim
    makes one limit-0 tsg_search per block. Driven from C threads (libtsg_shim_pattern.so:
    no GIL between calls, as goroutines have none), one per block of the set, each query
    over the next resident copy like the main line; libtsg coalesces the concurrent calls
    into one launch per batch (capi.cpp coalesced_search). Reported beside the batched main
    line (one tsg_search over all blocks)."""
    # (the caller threads get the idlest CPUs of the GPU's node, one per thread + 2, not the
    # main line's 8: more spinning threads than CPUs would time-slice the leader away)
    mask = os.sched_getaffinity(0)
    node = eng.numa_node(0)
    cpus = node_cpus(node) & all_cpus if node >= 0 else set()
    if len(cpus) > len(sets[0]) + 2:
        cpus = set(idlest(sorted(cpus), len(sets[0]) + 2))
    # limit 20 (the ingester's default): each block's call keeps its first 20 records; the
    # record count per query is the per-block searches' (one block per call)
    n20 = sum(eng.search_raw([b], pipe, limit=20)[0] for b in sets[0])
    try:
        if cpus and len(cpus) > len(mask):
            os.sched_setaffinity(0, cpus)
        eng.shim_pattern(sets, pipe, 16)  # warm (threads, per-thread scratch, pinned buffers)
        eng.shim_pattern(sets, pipe, 16, limit=20)
        if dist:
            dist.barrier()
        ns, nm = eng.shim_pattern(sets, pipe, args.shim_steps)
        ns20, nm20 = eng.shim_pattern(sets, pipe, args.shim_steps, limit=20)
    finally:
        os.sched_setaffinity(0, mask)
    assert all(x == nmatch for x in nm), "shim-pattern record count differs from the batched search"
    assert all(x == n20 for x in nm20), "shim-pattern limit-20 record count differs from the per-block searches"
    rate = entries * len(ns) / (sum(ns) / 1e9)
    return {"threads": len(sets[0]), "queries": len(ns), "entries_per_s": rate,
            "vs_batched": rate / batched if batched else None,
            "query_us": pct([x / 1e3 for x in ns]),
            "limit20": {"query_us": pct([x / 1e3 for x in ns20]), "records_per_query": n20,
                        "entries_per_s": entries * len(ns20) / (sum(ns20) / 1e9)},
            "note": "one C thread per block, each a tsg_search over its block (limit 0, and limit 20 "
                    "passed per block as Pipeline.Query carries it), per query; concurrent calls "
                    "coalesced into one launch (per-block caps under a limit); per-GPU rate"}


def cfg3_path(workdir, rank):
    return os.path.join(workdir, f"r{rank}cfg3")


def cfg3_generate(args, workdir, rank):
    """The config-3 block (one 5 M-entry block; the single-threaded writer takes ~1 min),
    started in a thread at bench start so it overlaps the config-2 legs."""
    import tempo_amd as T
    p = cfg3_path(workdir, rank)
    if not os.path.exists(os.path.join(p, "search.meta.json")):
        T.synth_search_block(p, args.cfg3_entries, seed=7000 + rank, profile=0, encoding=T.ENC_SNAPPY,
                             page_size=1024 * 1024)


def cfg3_leg(args, eng, pipe, workdir, rank, world, dist, sflags, gen_thread=None):
    """BASELINE config 3 on this GPU's share (200 blocks x 5 M over 8 GPUs = 25 x 5 M per
    GPU): one generated 5 M-entry block and device clones of it (tsg_block_clone: the
    clones share the host side), 125 M entries resident. Full scan: --cfg3-steps
    back-to-back queries (SURVEY.md 8(d)'s batched mode over a >= 100 M-entry resident
    set), kernel HIP events (dispatch-stamped) on every 8th; limit=20: the deterministic early exit."""
    import torch
    import tempo_amd as T
    t0 = time.time()
    p = cfg3_path(workdir, rank)
    if gen_thread is not None:
        gen_thread.join()
    cfg3_generate(args, workdir, rank)  # (no-op when the thread wrote it)
    gen_s = time.time() - t0  # (time still waited for the generator here)
    t0 = time.time()
    b0 = eng.open_block(p)
    blocks = [b0] + [b0.clone(eng) for _ in range(args.cfg3_blocks - 1)]
    load_s = time.time() - t0
    entries = sum(b.info()["entries"] for b in blocks)
    log(f"rank {rank}: cfg3 {len(blocks)} x {args.cfg3_entries} entries resident (gen {gen_s:.1f}s, "
        f"load+clone {load_s:.1f}s)")
    got, met = eng.search(blocks, pipe)
    for _ in range(2):
        eng.search_raw(blocks, pipe, flags=0)
    eng.kernel_times()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step = []
    for i in range(args.cfg3_steps):
        ts = time.perf_counter()
        eng.search_raw(blocks, pipe, flags=sflags if i % 8 == 4 else 0)
        step.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kns = eng.kernel_times() if sflags else []
    if dist:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    scan_bytes = met.scan_bytes
    kavg = sum(kns) / len(kns) if kns else 0
    ach = scan_bytes / kavg if kavg else None
    lim = []
    for i in range(23):
        ts = time.perf_counter()
        nl, metl = eng.search_raw(blocks, pipe, limit=20)
        if i >= 3:
            lim.append(time.perf_counter() - ts)
    # results kept for the oracle check after the timed legs (every copy is the same block)
    full_cols, full_met = eng.search_columns(blocks, pipe)
    lim_cols, lim_met = eng.search_columns(blocks, pipe, limit=20)
    nrep = len(blocks)

    def parity():
        from oracle import oracle as O
        q = oracle_query(QUERY)
        ob = O.Block(p)
        exp, omet, st = O.search([ob], **q)
        full_ok = st == 0 and columns_vs_oracle(full_cols, full_met, exp, omet, nrep)
        # limit 20 over the 25 copies: the sequential consumer (blocks in order) on the oracle
        lexp, lomet, lst = O.search([ob] * nrep, limit=20, **q)
        lim_ok = lst == 0 and len(lim_cols["start_ns"]) == len(lexp) and all(
            (int(lim_cols["block_idx"][i]), int(lim_cols["entry_idx"][i]), bytes(lim_cols["trace_id"][i]),
             int(lim_cols["start_ns"][i]), int(lim_cols["end_ns"][i]))
            == (m["block_idx"], m["entry_idx"], m["id"], m["start_ns"], m["end_ns"]) for i, m in enumerate(lexp)) and (
            lim_met.inspected_traces, lim_met.inspected_bytes, lim_met.inspected_blocks) == (
            lomet["traces_inspected"], lomet["bytes_inspected"], lomet["blocks_inspected"])
        return {"ok": bool(full_ok and lim_ok), "full_scan": bool(full_ok), "limit20": bool(lim_ok),
                "checked": f"full scan: all {len(full_cols['start_ns'])} matches of the {nrep} copies "
                           f"(every field, in order) + metrics vs the oracle on the block; limit 20: "
                           f"the oracle's sequential consumer over the {nrep} copies"}
    res = {
        "workload": f"config 3 per-GPU share: {len(blocks)} blocks x {args.cfg3_entries} entries "
                    f"(1 generated + {len(blocks) - 1} device clones), config-2 query",
        "entries_per_gpu": entries, "matches_full": len(got), "wait_for_generator_s": gen_s,
        "full_scan": {"queries": args.cfg3_steps, "entries_per_s": entries * args.cfg3_steps * world / elapsed,
                      "step_us": pct([x * 1e6 for x in step]), "kernel_us": pct([x / 1e3 for x in kns]),
                      "scan_bytes": scan_bytes, "achieved_gbps": ach,
                      "frac": ach / PEAK_HBM_GBPS if ach else None,
                      "regime": "hbm" if scan_bytes > 256 * 2**20 * 1.5 else "mall"},
        "limit20": {"matches": nl, "traces_inspected": metl.inspected_traces, "blocks_inspected": metl.inspected_blocks,
                    "time_to_first_20_us": pct([x * 1e6 for x in lim])},
    }
    for b in blocks:
        b.close()
    return res, parity


def cfg4_path(workdir, rank):
    return os.path.join(workdir, f"r{rank}cfg4")


def cfg4_generate(args, workdir, rank):
    """The config-4 block (the high-cardinality profile: ~unique http.url, 100-2000 B
    db.statement values; one block of --cfg4-entries), written in a thread at bench start."""
    import tempo_amd as T
    p = cfg4_path(workdir, rank)
    if not os.path.exists(os.path.join(p, "search.meta.json")):
        T.synth_search_block(p, args.cfg4_entries, seed=4000 + 97 * rank, profile=1, encoding=T.ENC_SNAPPY,
                             page_size=1024 * 1024)


CFG4_QUERIES = [
    ("statement+url", dict(tags={"db.statement": "from orders", "http.url": "/carts/"}, min_duration_ms=1)),
    ("statement_id_range", dict(tags={"db.statement": "where id = 77"}, start=QUERY["start"], end=QUERY["end"])),
    ("url_prefix", dict(tags={"http.url": "/api/v1/users/12"})),
    # a needle no value holds: MatchesBlock skips every block (blocksSkipped), from the
    # device dictionary pass (the host scan of the header's values took 24 ms)
    ("statement_absent", dict(tags={"db.statement": "qqzz"})),
]


def cfg4_leg(args, eng, workdir, rank, gen_thread=None):
    """BASELINE config 4 as config 2's size: --cfg4-blocks blocks of --cfg4-entries (10 x
    1 M = 10 M entries: one generated block and device clones of it, tsg_block_clone),
    high-cardinality tags (http.url, db.statement) with long values, ContainsTag semantics.
    Per query: the dictionary pass (every value of the searched keys tested for the needle:
    dict_stream_kernel over the value bytes, then the value-set bitmaps) and the scan; the
    block filter's tag half comes from the same pass. B_dict = the searched keys' dictionary
    bytes + offsets; the dictionary pass time = device sequence time (TIME_ALL events) - scan
    kernel time. step_over_device = step p50 / device p50 (host share of a query)."""
    import tempo_amd as T
    t0 = time.time()
    if gen_thread is not None:
        gen_thread.join()
    cfg4_generate(args, workdir, rank)
    gen_s = time.time() - t0
    t0 = time.time()
    p = cfg4_path(workdir, rank)
    b0 = eng.open_block(p)
    load1_s = time.time() - t0
    fb_gb = b0.info()["fb_bytes"] / 1e9
    blocks = [b0] + [b0.clone(eng) for _ in range(args.cfg4_blocks - 1)]
    load_s = time.time() - t0
    entries = sum(b.info()["entries"] for b in blocks)
    log(f"rank {rank}: cfg4 {len(blocks)} x {args.cfg4_entries} entries resident (gen wait {gen_s:.1f}s, "
        f"load {load1_s:.1f}s + clones {load_s - load1_s:.1f}s)")
    res = {"workload": f"config 4: {len(blocks)} blocks x {args.cfg4_entries} entries (1 generated + "
                       f"{len(blocks) - 1} device clones), high-cardinality profile (~unique http.url, "
                       f"100-2000 B db.statement)", "entries": entries, "load_s": load_s,
           "load_one_block_s": load1_s, "load_gb_per_s": fb_gb / load1_s if load1_s else None, "queries": {}}
    kept = {}
    for name, q in CFG4_QUERIES:
        pipe = T.Pipeline(T.SearchRequest(**q))
        # (the warmup with the timed steps' flags: a first TIME_ALL search of the dense query had
        # been one step in 20 at 5-6x the median, its first-use allocations inside the timing)
        n0, _ = eng.search_raw(blocks, pipe)
        eng.search_raw(blocks, pipe, flags=T.SEARCH_TIME_ALL)
        ts_all, dict_ns, scan_ns, steps = [], [], [], []
        met = None
        for i in range(args.cfg4_steps):
            ts = time.perf_counter()
            n, met = eng.search_raw(blocks, pipe, flags=T.SEARCH_TIME_ALL)
            steps.append(time.perf_counter() - ts)
            assert n == n0
            ts_all.append(met.kernel_ns)
            scan_ns.append(met.scan_kernel_ns)
            dict_ns.append(met.kernel_ns - met.scan_kernel_ns)
        if os.environ.get("TSG_PROF"):  # (host phases per query)
            from tempo_amd import tsg as _tsg
            _tsg.lib().tsgx_prof_flush(name.encode())
        b_dict = met.device_bytes_read - met.scan_bytes
        dmed = sorted(dict_ns)[len(dict_ns) // 2]
        smed = sorted(scan_ns)[len(scan_ns) // 2]
        amed = sorted(ts_all)[len(ts_all) // 2]
        spmed = sorted(steps)[len(steps) // 2]
        res["queries"][name] = {
            "query": q, "matches": n0, "blocks_inspected": met.inspected_blocks, "blocks_skipped": met.skipped_blocks,
            "step_us": pct([x * 1e6 for x in steps]),
            "entries_per_s": entries / spmed,
            "device_us": pct([x / 1e3 for x in ts_all]),
            "step_over_device": spmed * 1e9 / amed if amed else None,
            "dict_pass_us": pct([x / 1e3 for x in dict_ns]), "scan_us": pct([x / 1e3 for x in scan_ns]),
            "b_dict": b_dict, "scan_bytes": met.scan_bytes,
            "dict_gbps": b_dict / dmed if dmed else None,
            "dict_frac": b_dict / dmed / PEAK_HBM_GBPS if dmed else None,
            "scan_gbps": met.scan_bytes / smed if smed else None,
        }
        if args.parity:
            kept[name] = (q, eng.search_columns(blocks, pipe))
    nrep = len(blocks)
    for b in blocks:
        b.close()

    def parity():
        from oracle import oracle as O
        ob = O.Block(p)
        out = {}

        def one(name):
            q, (cols, gmet) = kept[name]
            exp, omet, st = O.search([ob], **oracle_query(q))
            out[name] = bool(st == 0 and columns_vs_oracle(cols, gmet, exp, omet, nrep))
        parallel(one, list(kept))
        return {"ok": all(out.values()), "queries": out,
                "checked": f"every query: all matches of the {nrep} copies (every field, in order) and the "
                           f"metrics (blocks skipped / inspected, traces, bytes) vs the oracle on the block"}
    return res, parity if args.parity else None


def cfg5_dir(shared):
    return os.path.join(shared, "cfg5")


def cfg5_generate(args, shared, rank, world):
    """Config-5 v2 blocks (synthetic ids, bloom fp 0.01 with 100 KiB shards, index over
    1 MiB data pages), written into a directory every rank of this node reads: rank r
    writes blocks i = r mod world (each with its ids beside it as ids.npy)."""
    import numpy as np
    import tempo_amd as T
    d = cfg5_dir(shared)
    os.makedirs(d, exist_ok=True)

    def one(i):
        p = os.path.join(d, f"v2_{i:03d}")
        if not os.path.exists(os.path.join(p, "ids.npy")):
            ids = T.synth_v2_block(p, args.cfg5_objects, seed=9000 + i)
            np.save(os.path.join(p, "ids.tmp.npy"), ids)
            os.replace(os.path.join(p, "ids.tmp.npy"), os.path.join(p, "ids.npy"))
    mine = [i for i in range(args.cfg5_blocks) if i % world == rank]
    nth = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    for k in range(0, len(mine), nth):
        parallel(one, mine[k:k + nth])


def cfg5_leg(args, eng, shared, rank, world, dist, gen_thread=None):
    """BASELINE config 5: batched trace-ID lookup, --cfg5-probes ids (half present in some
    block, half random) against --cfg5-blocks v2 blocks (bloom + sorted index; every block on
    every rank), the ids sharded over the ranks (shard.shard_ids: no exchange on the data
    path). value = probes over all ranks / the slowest rank's device time (tsg_lookup_ids'
    event pair around slab build + count + write: ids resident, hits in HBM); host_e2e adds
    moving ids in and hits out (PCIe). N > 1: the per-rank hit tables gathered to rank 0 over
    RCCL (shard.distributed_lookup on cuda) once, timed."""
    import numpy as np
    import torch
    import tempo_amd as T
    from tempo_amd import shard
    if gen_thread is not None:
        gen_thread.join()
    cfg5_generate(args, shared, rank, world)
    if dist:
        dist.barrier()
    d = cfg5_dir(shared)
    paths = [os.path.join(d, f"v2_{i:03d}") for i in range(args.cfg5_blocks)]
    present = np.concatenate([np.load(os.path.join(p, "ids.npy")) for p in paths])
    rng = np.random.default_rng(5)
    half = args.cfg5_probes // 2
    probes = np.concatenate([present[rng.integers(0, len(present), half)],
                             rng.integers(0, 256, (args.cfg5_probes - half, 16), dtype=np.uint8)])
    probes = np.ascontiguousarray(probes[rng.permutation(len(probes))])
    del present
    sl = shard.shard_ids(len(probes), world, rank)
    mine = np.ascontiguousarray(probes[sl.start:sl.stop])
    old = os.environ.get("TSG_V2_NO_DATA")
    os.environ["TSG_V2_NO_DATA"] = "1"  # (the lookup reads bloom + index only)
    t0 = time.time()
    try:
        blocks = parallel(eng.open_v2block, paths)
    finally:
        if old is None:
            os.environ.pop("TSG_V2_NO_DATA", None)
        else:
            os.environ["TSG_V2_NO_DATA"] = old
    load_s = time.time() - t0
    hits, _ = eng.lookup(blocks, mine)  # warm
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    walls, kns = [], []
    t0 = time.perf_counter()
    for _ in range(args.cfg5_steps):
        ts = time.perf_counter()
        nh, kns_i = eng.lookup_raw(blocks, mine)  # (the ABI call as a Go caller makes it: no conversion)
        walls.append(time.perf_counter() - ts)
        kns.append(kns_i)
    elapsed = time.perf_counter() - t0
    kmed = sorted(kns)[len(kns) // 2]
    if dist:
        t = torch.tensor([elapsed, float(kmed)], dtype=torch.float64, device=RED_DEVICE)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmed = float(t[0].item()), float(t[1].item())
    res = {"workload": f"config 5: {args.cfg5_probes} probe ids (50 % present) x {args.cfg5_blocks} v2 blocks "
                       f"of {args.cfg5_objects} objects, ids sharded over {world} rank(s)",
           "probes_per_rank": len(mine), "steps": args.cfg5_steps, "load_s": load_s,
           "value": args.cfg5_probes / (kmed / 1e9), "unit": "probes/s",
           "device_ms": kmed / 1e6, "probe_block_pairs_per_s": args.cfg5_probes * args.cfg5_blocks / (kmed / 1e9),
           "host_e2e": {"probes_per_s": args.cfg5_probes * args.cfg5_steps / elapsed,
                        "step_ms": pct([x * 1e3 for x in walls]),
                        "note": "tsg_lookup_ids + tsg_lookup_result_free on pageable ids (staged through "
                                "pinned chunks), hit columns left in the result's pinned arrays"},
           "hits_rank0": int(len(hits)),
           "requests_per_probe": "6.3 random 64-B slab reads (PMC FETCH_SIZE, profiles/r03_lookup)"}
    if dist:
        t0 = time.perf_counter()
        allhits = shard.distributed_lookup(lambda x: eng.lookup(blocks, x)[0], probes, device=RED_DEVICE)
        torch.cuda.synchronize()
        res["rccl_gather" if not SHARED_GPU else "gloo_gather"] = {
            "s": time.perf_counter() - t0, "hits": int(len(allhits)) if allhits is not None else None,
            "note": "lookup of every rank's slice + dist.gather of the hit tables to rank 0 over RCCL "
                    "(nccl backend, cuda tensors)" if not SHARED_GPU else
                    "ranks share one GPU (--ranks-share-gpu): the hit tables gathered over gloo; the RCCL "
                    "gather is skipped (RCCL needs one GPU per rank)"}
    for b in blocks:
        b.close()
    check = probes[:20_000] if rank == 0 else None
    got_check = hits[hits[:, 0] < 20_000] if rank == 0 else None

    def parity():
        from oracle import oracle as O
        ob = [O.V2Block(p) for p in paths]
        nthr = max(1, min(16, len(os.sched_getaffinity(0))))
        rc, exp = O.lookup(ob, check, nthreads=nthr)
        ok = rc == 0 and np.array_equal(got_check, np.array(exp, dtype=np.int64).reshape(-1, 5))
        # the CPU baseline on the same host: the oracle's lookup (pthreads over probes)
        cs = probes[:200_000]
        t0 = time.perf_counter()
        O.lookup(ob, cs, nthreads=nthr)
        dt = time.perf_counter() - t0
        return {"ok": bool(ok), "checked": f"every hit (id, block, record, start, length) of the first "
                                           f"{len(check)} probes vs the oracle's lookup",
                "cpu_baseline": {"value": len(cs) / dt, "unit": "probes/s", "cores": nthr, "kind": "port",
                                 "sample": f"first {len(cs)} probes x all {len(paths)} blocks, oracle lookup "
                                           f"(oracle/tsg_oracle.c, {nthr} threads), {dt:.2f} s"}}
    return res, parity if (args.parity and rank == 0) else None


def merge_leg(args, eng, base, pipe, rank, world, dist):
    """N > 1: the query as the frontend serves it (modules/frontend/searchsharding.go:32-125):
    every rank searches its block shard (full scan, the config-2 query), packs its ordered
    match list into a wire buffer (tsg_result_pack), rank 0 gathers them
    (tempo_amd.shard.distributed_search_packed) and merges them in libtsg (tsg_wire_merge). A few hundred records per rank: gathered on the host over a gloo group
    (north_star: "host-merged where that is cheaper"; the RCCL form of the same gather is
    covered by the packed-gather tests). Latency per query is the max over ranks."""
    from datetime import timedelta

    import torch
    from tempo_amd import shard
    try:
        g = dist.new_group(backend="gloo", timeout=timedelta(seconds=120))
        nb = len(base) * world
        everything = 1 << 30  # (full scan: the frontend merge keeps every distinct trace)
        local = lambda: eng.search_wire(base, pipe)  # noqa: E731  (tsg_result_pack: no per-record Python)
        merged = shard.distributed_search_packed(local, everything, nb, device="cpu", group=g, columns=True)
        dist.barrier(group=g)
        ts = []
        for _ in range(args.merge_steps):
            t0 = time.perf_counter()
            merged = shard.distributed_search_packed(local, everything, nb, device="cpu", group=g, columns=True)
            dist.barrier(group=g)
            ts.append(time.perf_counter() - t0)
        tt = torch.tensor([sum(ts)], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=g)
        res = {"queries": args.merge_steps, "ranks": world, "step_us": pct([x * 1e6 for x in ts]),
               "entries_per_s": len(base) * args.entries * world * args.merge_steps / float(tt.item()),
               "transport": "gloo (host) gather of packed records to rank 0, then merge"}
        if rank == 0:
            res["merged_traces"] = len(merged)
            res["inspected_traces"] = merged.metrics.inspected_traces
            res["block_errors"] = sum(1 for x in merged.block_status if x)
        # the merged query through shared memory (the node's ranks: tsg_shm_put / tsg_shm_merge):
        # each timed step = this rank's full scan + its response into its slot; rank 0's step also
        # waits for every rank and merges (queries back to back: no barrier between them)
        try:
            shm = shard.ShmGather("tsg_bench_%s" % os.environ.get("MASTER_PORT", "0"), world, rank, group=g)
            try:
                # this rank's part alone (search + pack, no gather): what the merged step adds is
                # the step minus this (both ranks on one GPU under --ranks-share-gpu: their scans
                # share it, so this is measured with the other rank scanning too)
                dist.barrier(group=g)
                tl = []
                for _ in range(args.merge_steps):
                    t0 = time.perf_counter()
                    local()
                    tl.append(time.perf_counter() - t0)
                for _ in range(3):
                    m3 = shm.query(local(), everything, nb)
                dist.barrier(group=g)
                ts3 = []
                for _ in range(args.merge_steps):
                    t0 = time.perf_counter()
                    m3 = shm.query(local(), everything, nb)
                    ts3.append(time.perf_counter() - t0)
                dist.barrier(group=g)
                tt3 = torch.tensor([sum(ts3)], dtype=torch.float64)
                dist.all_reduce(tt3, op=dist.ReduceOp.MAX, group=g)
                res["shm"] = {"step_us": pct([x * 1e6 for x in ts3]), "local_search_wire_us": pct([x * 1e6 for x in tl]),
                              "entries_per_s": len(base) * args.entries * world * args.merge_steps / float(tt3.item()),
                              "transport": "shared memory (/dev/shm) slots per rank, merged in place on rank 0"}
                if rank == 0:
                    res["shm"]["same_as_gloo"] = bool(len(m3) == len(merged) and (m3.recs == merged.recs).all())
            finally:
                shm.close()
        except Exception as e:  # noqa: BLE001
            res["shm"] = {"error": repr(e)}
        if SHARED_GPU:
            res["rccl"] = "skipped: shared device (--ranks-share-gpu: RCCL needs one GPU per rank)"
            return res
        # the same gather as cuda byte tensors over the default (nccl = RCCL over xGMI) group
        m2 = shard.distributed_search_packed(local, everything, nb, device="cuda", columns=True)
        dist.barrier()
        ts2 = []
        for _ in range(args.merge_steps):
            t0 = time.perf_counter()
            m2 = shard.distributed_search_packed(local, everything, nb, device="cuda", columns=True)
            dist.barrier()
            ts2.append(time.perf_counter() - t0)
        res["rccl"] = {"step_us": pct([x * 1e6 for x in ts2]),
                       "transport": "RCCL gather of the packed records (cuda uint8 tensors) to rank 0, then merge"}
        if rank == 0:
            res["rccl"]["same_as_gloo"] = bool(len(m2) == len(merged) and (m2.recs == merged.recs).all())
        return res
    except Exception as e:  # (the main line above is already measured; report, do not fail)
        return {"error": repr(e)}


def main():
    args = parse()
    re = rank_env(args)
    if re is None:  # --gpus N, no torchrun around us: start the ranks (nothing has touched a GPU)
        sys.exit(launch_ranks(args, sys.argv[1:]))
    rank, world, local = re
    global RED_DEVICE, SHARED_GPU
    if args.ranks_share_gpu and world > 1:
        # a rehearsal of the N-rank path on a 1-GPU lease: every rank on device 0, collectives
        # over gloo (the RCCL legs report "skipped: shared device")
        SHARED_GPU, RED_DEVICE, local = True, "cpu", 0
    if args.cfg3 is None:
        args.cfg3 = 1  # (config 3 is an 8-GPU config: every rank runs its share)
    if args.cfg4 is None:
        args.cfg4 = 1 if world == 1 else 0
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if SHARED_GPU else "nccl")
    torch.cuda.set_device(local)

    import tempo_amd as T

    workdir = args.workdir or tempfile.mkdtemp(prefix="tsg_bench_", dir="/tmp")
    os.makedirs(workdir, exist_ok=True)
    # files every rank of the node reads (config 5's replicated v2 blocks): one directory per run
    shared = os.path.join(args.workdir, "shared") if args.workdir else os.path.join(
        "/tmp", "tsg_bench_shared_%s_%s" % (os.environ.get("MASTER_PORT", "solo"), os.environ.get(
            "TORCHELASTIC_RUN_ID", os.getppid() if world > 1 else os.getpid())))
    os.makedirs(shared, exist_ok=True)
    threads = min(args.blocks, max(1, min(16, (os.cpu_count() or 8)) // max(1, min(world, 8))))
    gens = {}
    if args.cfg3:
        gens["cfg3"] = threading.Thread(target=cfg3_generate, args=(args, workdir, rank), daemon=True)
    if args.cfg4:
        gens["cfg4"] = threading.Thread(target=cfg4_generate, args=(args, workdir, rank), daemon=True)
    if args.cfg5:
        gens["cfg5"] = threading.Thread(target=cfg5_generate, args=(args, shared, rank, world), daemon=True)
    for th in gens.values():
        th.start()
    t0 = time.time()
    paths = gen_blocks(workdir, rank, args.blocks, args.entries, threads)
    log(f"rank {rank}: generated {args.blocks} x {args.entries} entries in {time.time() - t0:.1f}s")
    # The config-3/4/5 generator threads (started at bench start, beside this set's synthesis)
    # finish here, before the engine opens anything: no load or timed leg shares the host's
    # CPUs with them, and the GPU is not left idle between the warmup and the timed steps.
    t0 = time.time()
    for th in gens.values():
        th.join()
    log(f"rank {rank}: waited {time.time() - t0:.1f}s for the cfg3/4/5 generators")

    streams = max(1, args.streams) if args.concurrent_steps else 1
    eng = T.Engine(devices=[local])
    t0 = time.time()
    base = parallel(eng.open_block, paths)
    load_s = time.time() - t0
    infos = [b.info() for b in base]
    entries = sum(i["entries"] for i in infos)
    fb_bytes = sum(i["fb_bytes"] for i in infos)
    dev_bytes = sum(i["device_bytes"] for i in infos)
    log(f"rank {rank}: loaded {entries} entries ({fb_bytes / 1e9:.2f} GB flatbuffer) in {load_s:.1f}s, "
        f"{dev_bytes / 1e9:.2f} GB resident")
    # disjoint resident copies of the set: the rotation's working set is sets x the set
    sets = [tuple(base)] + [tuple(b.clone(eng) for b in base) for _ in range(max(1, args.sets) - 1)]
    if len(sets) > 1:
        log(f"rank {rank}: {len(sets)} resident copies of the set ({len(sets) * dev_bytes / 1e9:.2f} GB)")

    all_cpus = os.sched_getaffinity(0)
    # the CPU baselines' threads: this GPU's share of its node's CPUs (an MI355X node: 8 GPUs;
    # nproc / 8 = 32 on the 256-CPU boxes), at least 16, at most the CPUs this process may use
    cpu_threads = args.cpu_threads or max(1, min(len(all_cpus), max((os.cpu_count() or 8) // 8, min(16, len(all_cpus)))))
    if args.pin == "auto":
        # the step polls a completion word and copies its records from pinned host memory:
        # both are served faster from the GPU's own socket (profiles/r01_host).
        # After loading (which uses many threads): 8 CPUs of that node, a slice per local rank.
        node = eng.numa_node(0)
        cpus = sorted(node_cpus(node) & os.sched_getaffinity(0)) if node >= 0 else []
        if cpus:
            # a slice of the node per local rank, then its 8 idlest CPUs
            lws = int(os.environ.get("LOCAL_WORLD_SIZE", world))
            per = max(8, len(cpus) // max(1, lws))
            k = (local * per) % len(cpus)
            mine = set(idlest(cpus[k:k + per] or cpus, 8))
            os.sched_setaffinity(0, mine)
        log(f"rank {rank}: GPU NUMA node {node}, search thread on CPUs {sorted(mine)}" if cpus else
            f"rank {rank}: GPU NUMA node unknown, not pinned")
    req = T.SearchRequest(tags=QUERY["tags"], min_duration_ms=QUERY["min_duration_ms"],
                          max_duration_ms=QUERY["max_duration_ms"], start=QUERY["start"], end=QUERY["end"])
    pipe = T.Pipeline(req)
    got, met = eng.search(base, pipe)  # full result once (parity check against the oracle below)
    for s in sets[1:]:
        g2, _ = eng.search(s, pipe)
        assert [(m.block_idx, m.entry_idx, m.trace_id) for m in g2] == [(m.block_idx, m.entry_idx, m.trace_id)
                                                                        for m in got], "clone differs"
    # HIP events on the search kernel of every --events-th timed step, on the library's
    # stream, stamped from the kernel's own dispatch packet (hipExtLaunchKernel: what
    # rocprofv3's kernel trace measures); read after the timed region (the search does not
    # wait for them). Not every step carries a pair: recording one costs the host time.
    sflags = T.SEARCH_TIME_DEFER if args.events else 0
    ev_phase = args.events // 2  # (sampled steps: i % events == events // 2, never the first step)

    def timed(nsteps, rot):
        step_s = []
        t0 = time.perf_counter()
        for i in range(nsteps):  # (tsg_search is synchronous: results are on the host when it returns)
            ts = time.perf_counter()
            eng.search_raw(sets[i % rot], pipe, flags=sflags if args.events and i % args.events == ev_phase else 0,
                           metrics=False)
            step_s.append(time.perf_counter() - ts)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, step_s

    # Python's cyclic GC stays off through the timed legs (re-enabled before the CPU
    # baselines): a collection pass over this process's heap is host noise that the
    # library's real caller, a Go querier, does not have. Collected BEFORE the warmup, so
    # that the warmup steps run right before the timed ones (a GPU left idle for the tens of
    # milliseconds a collection takes runs its next kernel ~2x slower)
    gc.collect()
    gc.disable()
    eng.kernel_times()  # (drain)
    res0 = eng.resident_counters()
    for i in range(max(args.warmup, len(sets))):
        eng.search_raw(sets[i % len(sets)], pipe, flags=0)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed, step_s = timed(args.steps, len(sets))
    scan_ns = eng.kernel_times() if args.events else []
    if dist:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        te = torch.tensor([entries], dtype=torch.float64, device=RED_DEVICE)
        dist.all_reduce(te, op=dist.ReduceOp.SUM)
        total_entries = int(te.item())
    else:
        total_entries = entries

    res1 = eng.resident_counters()
    # the main line served by the resident search kernel (pool.hip, TSG_RESIDENT): each query's
    # device time is its span on the device (the first workgroup to read it .. the last to store
    # its count, s_memrealtime), not a dispatch's duration (there is none per query)
    resident = res1["queries"] - res0["queries"] >= args.steps
    kernel_name = "search_resident_kernel<3, true, true, %s>" % KERNEL.rsplit(", ", 1)[1].rstrip(">") \
        if resident and KERNEL.startswith("search_pool_kernel") else KERNEL
    ms_per_step = elapsed / args.steps * 1e3
    value = total_entries * args.steps / elapsed
    scan_avg_ns = sum(scan_ns) / len(scan_ns) if scan_ns else 0
    scan_bytes = met.scan_bytes
    achieved = scan_bytes / scan_avg_ns if scan_avg_ns else None  # bytes/ns == GB/s
    regime = "hbm" if len(sets) * scan_bytes > 256 * 2**20 * 1.5 else "mall"
    # (the PMC figure of this layout: the pool kernels' 11 B/entry columns, round 4 on)
    traffic, traffic_src = pmc_traffic(f"blocks={args.blocks},entries={args.entries},sets={len(sets)},layout=ds",
                                       kernel_name)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "entries/s",
        "n_gpus": 1 if SHARED_GPU else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 integer columns",
        "data": "synthetic (seeded SURVEY.md §8d generator, snappy 1 MiB pages)",
        "config": {
            "workload": "cfg2: 10M-entry block set per GPU, 3-tag AND + min/max duration + time range, "
                        "full scan (limit 0), ordered match list",
            "blocks_per_gpu": args.blocks, "entries_per_block": args.entries, "entries_per_gpu": entries,
            "resident_sets": len(sets), "query": QUERY, "limit": 0, "matches_per_gpu": len(got),
            "parallelism": f"block-sharded x{world}" + (" ranks on ONE GPU (--ranks-share-gpu rehearsal)"
                                                         if SHARED_GPU else ""),
        },
        "achieved_hbm_gbps": achieved,
        "roofline": {
            "bound": "hbm", "kernel": kernel_name, "achieved": achieved, "peak": PEAK_HBM_GBPS,
            "device_time": ("per-query span in the resident kernel (first workgroup to read the query .. "
                            "last workgroup's count stored; s_memrealtime, 100 MHz)") if resident else
                           "dispatch timestamps of the launch (AQL profiling / hipExtLaunchKernel events)",
            "unit": "GB/s", "frac": achieved / PEAK_HBM_GBPS if achieved else None,
            "regime": regime,
            "regime_note": (f"each step searches the next of {len(sets)} disjoint resident copies of the set "
                            f"({len(sets)} x {scan_bytes / 1e6:.0f} MB of filter columns per rotation > the "
                            f"256 MiB Infinity Cache)" if len(sets) > 1 else
                            "the same set every step: its filter columns stay in the 256 MiB Infinity Cache"),
            "traffic": traffic, "traffic_measured_in_run": False,
            "traffic_source": traffic_src, "bytes_per_launch": scan_bytes, "avg_launch_us": scan_avg_ns / 1e3,
            "bytes_per_entry": round(scan_bytes / entries, 3),
        },
        "load_s": load_s,
        "load_gb_per_s": fb_bytes / load_s / 1e9 if load_s else None,
        "flatbuffer_gb_per_gpu": fb_bytes / 1e9,
    }
    out["latency_us"] = {"step": pct([x * 1e6 for x in step_s]), "kernel": pct([x / 1e3 for x in scan_ns])}
    out["resident"] = {"main_line": resident, **{k: res1[k] - res0[k] for k in res1}}

    if args.mall_steps and len(sets) > 1:
        # the same set every step: its columns stay in the Infinity Cache (round 1's regime)
        e2, s2 = timed(args.mall_steps, 1)
        k2 = eng.kernel_times() if args.events else []
        a2 = scan_bytes / (sum(k2) / len(k2)) if k2 else None
        out["mall"] = {"steps": args.mall_steps, "entries_per_s": entries * args.mall_steps / e2,
                       "step_us": pct([x * 1e6 for x in s2]), "kernel_us": pct([x / 1e3 for x in k2]),
                       "achieved_gbps": a2, "frac": a2 / PEAK_HBM_GBPS if a2 else None}

    if args.batch_queries:
        out["batched"] = batch_leg(args, eng, sets, pipe, entries, scan_bytes, len(got))

    if args.limit_steps:
        # SURVEY.md §8(d) config-3 mode on this rank's set: limit=20 (ingester default),
        # the deterministic early-exit rule, same query; reported beside the full scan
        for _ in range(3):
            eng.search_raw(base, pipe, limit=20)
        eng.kernel_times()
        ls = []
        for i in range(args.limit_steps):
            ts = time.perf_counter()
            nl, metl = eng.search_raw(sets[i % len(sets)], pipe, limit=20,
                                      flags=sflags if args.events and i % args.events == ev_phase else 0)
            ls.append(time.perf_counter() - ts)
        lk = eng.kernel_times() if args.events else []
        out["limit20"] = {"steps": args.limit_steps, "matches": nl, "traces_inspected": metl.inspected_traces,
                          "step_us": pct([x * 1e6 for x in ls]), "kernel_us": pct([x / 1e3 for x in lk]),
                          "entries_per_s": entries / (sum(ls) / len(ls))}

    if args.shim_steps:
        out["shim"] = shim_leg(args, eng, sets, pipe, entries, len(got), value / max(1, world), dist, all_cpus)

    if args.concurrent_steps and streams > 1:
        out["concurrent"] = concurrent_leg(args, base, pipe, streams, entries, dist, world, local)

    checks = {}
    if args.cfg3:
        out["cfg3"], checks["cfg3"] = cfg3_leg(args, eng, pipe, workdir, rank, world, dist, sflags)

    if args.cfg4:
        # a dense config-4 query assembles ~1.85 M records on the host (the library's parallel
        # fill, on the calling thread's CPUs): this leg gets 16 CPUs of the GPU's node (the
        # job's CPU share), the latency legs keep their 8 idlest
        narrow = os.sched_getaffinity(0)
        node = eng.numa_node(0)
        wide = sorted(node_cpus(node) & all_cpus) if node >= 0 else []
        if args.pin == "auto" and len(wide) > len(narrow):
            os.sched_setaffinity(0, set(idlest(wide, 16)))
        try:
            out["cfg4"], checks["cfg4"] = cfg4_leg(args, eng, workdir, rank)
            out["cfg4"]["host_cpus"] = len(os.sched_getaffinity(0))
        finally:
            os.sched_setaffinity(0, narrow)

    if args.cfg5:
        out["cfg5"], checks["cfg5"] = cfg5_leg(args, eng, shared, rank, world, dist)

    if world > 1 and args.merge_steps:
        out["merge"] = merge_leg(args, eng, base, pipe, rank, world, dist)

    cfg1_cpu = None
    if args.cfg1 and rank == 0:
        out["cfg1"], cfg1_cpu = cfg1_leg(args, eng, base[0], paths[0], args.cfg1_steps)

    for s in sets:
        for b in s:
            b.close()
    eng.close()
    gc.enable()
    os.sched_setaffinity(0, all_cpus)  # (the host checks and CPU baselines get the whole host share back)
    if args.parity:
        # the oracle checks of the cfg3/cfg4/cfg5 legs (rank 0 reports; every rank checks its own share)
        jobs = {k: v for k, v in checks.items() if v is not None}
        t0 = time.time()
        par = run_parity(jobs)
        log(f"rank {rank}: parity {', '.join('%s=%s' % (k, v.get('ok')) for k, v in par.items())} "
            f"in {time.time() - t0:.1f}s")
        for k, v in par.items():
            if k == "cfg5" and "cpu_baseline" in v:
                out[k]["cpu_baseline"] = v.pop("cpu_baseline")
            out[k]["parity"] = v
        if dist:
            ok = torch.tensor([int(all(v.get("ok") for v in par.values()))], dtype=torch.int32)
            g = dist.new_group(backend="gloo")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=g)
            out["parity_all_ranks"] = bool(ok.item())
    if rank == 0 and world == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baselines(paths, got, cpu_threads, oracle_threads=cpu_threads)
    if cfg1_cpu is not None:
        try:
            out["cfg1"]["parity"] = cfg1_cpu()
        except Exception as e:  # noqa: BLE001  (reported; the timed figures stand)
            out["cfg1"]["parity"] = {"ok": False, "error": repr(e)}

    if rank == 0:
        out["summary"] = summary(out)  # (last: a reader that keeps only the line's tail still sees it)
        print(json.dumps(out), flush=True)
    if not args.keep and not args.workdir:
        shutil.rmtree(workdir, ignore_errors=True)
        if rank == 0:
            shutil.rmtree(shared, ignore_errors=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
