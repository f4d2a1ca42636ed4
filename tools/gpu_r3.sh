#!/bin/bash
# Round-3 GPU-box session: stages chosen by $1 (comma list). Every GPU step runs under its
# own timeout; the script stops at the first failure (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-merge,live,probe,bench}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 test failures (no crash)

if has merge; then  # CPU only (a fresh process, no device touched): the merge path's host cost
  TSG_MERGE_BOUND_MS=100 timeout -k 10 300 python -u -m pytest tests/test_shard_gloo.py -x -v -s -p no:cacheprovider \
    -k "million or native_merge or wire" > gpurun_out/merge_perf.log 2>&1
  rc=$?; echo "merge perf rc=$rc"; grep -E "best|passed|failed" gpurun_out/merge_perf.log | tail -3
  ok_rc $rc || exit $rc
fi
if has live; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_live.py tests/test_gpu_multiproc.py tests/test_gpu_proto.py \
    tests/test_gpu_search.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_live.log 2>&1
  rc=$?; echo "pytest live rc=$rc"; tail -15 gpurun_out/pytest_live.log
  ok_rc $rc || exit $rc
fi
if has core; then  # the search-kernel tests (pool/static kernels, limits, coalescer, configs, damaged blocks)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_search.py tests/test_gpu_coalesce.py \
    tests/test_gpu_configs.py tests/test_gpu_damaged.py tests/test_gpu_lookup.py tests/test_gpu_dict_stream.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_core.log 2>&1
  rc=$?; echo "pytest core rc=$rc"; tail -4 gpurun_out/pytest_core.log
  [ $rc -eq 0 ] || exit $rc
fi
if has gputest; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  ok_rc $rc || exit $rc
fi
if has probe; then
  hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o gpurun_out/launch_probe || exit 1
  timeout -k 10 120 gpurun_out/launch_probe > gpurun_out/launch_probe.json 2>&1
  rc=$?; echo "probe rc=$rc"; cat gpurun_out/launch_probe.json
  [ $rc -eq 0 ] || exit $rc
fi
if has lookup; then
  T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
  timeout -k 10 300 $T tests/test_gpu_lookup.py tests/test_gpu_configs.py -k "lookup or find or cfg5 or fixture or blocks or range or devices" \
    > gpurun_out/lk_tests.log 2>&1
  rc=$?; echo "lookup tests rc=$rc"; tail -3 gpurun_out/lk_tests.log
  [ $rc -eq 0 ] || exit $rc
  for d in 0 1; do
    TSG_LK_PAIR=$d timeout -k 10 400 python tools/bench_lookup.py --cpu-sample 0 ${LK_ARGS:-} > gpurun_out/lookup_pair$d.json 2> gpurun_out/lookup_pair$d.err
    rc=$?; echo "lookup bench pair=$d rc=$rc"; cut -c1-260 gpurun_out/lookup_pair$d.json
    [ $rc -eq 0 ] || exit $rc
  done
fi
if has lkprof; then  # config-5 lookup: per-kernel times and line traffic of the count pass
  export TMPDIR=/tmp
  LKA="--cpu-sample 0 --check 2000 --steps 3"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof -o run --output-format csv -- \
    python3 tools/bench_lookup.py $LKA > gpurun_out/lkprof.json 2> gpurun_out/lkprof.err
  rc=$?; echo "lk rocprof rc=$rc"; cat gpurun_out/lkprof/run_kernel_stats.csv 2>/dev/null || find gpurun_out/lkprof -name "*stats.csv"
  [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/lkpmc_$c -o run --output-format csv -- \
      python3 tools/bench_lookup.py $LKA > gpurun_out/lkpmc_$c.json 2> gpurun_out/lkpmc_$c.err
    rc=$?; echo "lk pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/lkpmc_FETCH_SIZE gpurun_out/lkpmc_WRITE_SIZE --match lookup \
    --workload "lookup,blocks=200,objects=100000,probes=10000000" --source "tools/gpu_r3.sh lkprof" | tee gpurun_out/lkpmc_summary.txt
fi
if has scanprobe; then
  hipcc -O3 --offload-arch=gfx950 tools/scan_probe.hip -o gpurun_out/scan_probe || exit 1
  timeout -k 10 180 gpurun_out/scan_probe > gpurun_out/scan_probe.json 2>&1
  rc=$?; echo "scan probe rc=$rc"; cat gpurun_out/scan_probe.json
  [ $rc -eq 0 ] || exit $rc
  PROBE_RAND=1 timeout -k 10 180 gpurun_out/scan_probe > gpurun_out/scan_probe_rand.json 2>&1
  rc=$?; echo "scan probe rand rc=$rc"; cat gpurun_out/scan_probe_rand.json
  [ $rc -eq 0 ] || exit $rc
fi
if has stamps; then
  TSG_STAMPS=1 timeout -k 10 600 python bench.py --steps 6 --warmup 2 --cpu-baseline 0 --cfg3 0 --concurrent-steps 0 \
    --mall-steps 0 ${BENCH_ARGS:-} > gpurun_out/stamps.json 2> gpurun_out/stamps.err
  rc=$?; echo "stamps rc=$rc"; grep "stamps" gpurun_out/stamps.err | tail -6
  [ $rc -eq 0 ] || exit $rc
fi
if has ab; then  # the static-run kernel vs the claim-based pool kernel, same box, same legs
  for st in 1 0; do
    TSG_POOL_STATIC=$st timeout -k 10 400 python bench.py --steps 400 --cpu-baseline 0 --concurrent-steps 0 --cfg4 0 \
      --mall-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_static$st.json 2> gpurun_out/ab_static$st.err
    rc=$?; echo "ab static=$st rc=$rc"; tail -2 gpurun_out/ab_static$st.err
    [ $rc -eq 0 ] || exit $rc
    TSG_POOL_STATIC=$st TSG_STAMPS=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --cpu-baseline 0 --cfg3 0 \
      --concurrent-steps 0 --cfg4 0 --shim-steps 0 --limit-steps 4 --mall-steps 0 > gpurun_out/stamps_static$st.json 2> gpurun_out/stamps_static$st.err
    rc=$?; echo "stamps static=$st rc=$rc"; grep "stamps" gpurun_out/stamps_static$st.err | tail -4
    [ $rc -eq 0 ] || exit $rc
  done
  python3 - <<'PY'
import json
for st in (1, 0):
    d = json.load(open(f"gpurun_out/ab_static{st}.json"))
    print(st, "value", round(d["value"] / 1e9, 1), "frac", round(d["roofline"]["frac"], 3), "kernel", d["latency_us"]["kernel"],
          "lim20", d["limit20"]["kernel_us"]["p50"], d["limit20"]["step_us"]["p50"],
          "cfg3", d["cfg3"]["full_scan"]["kernel_us"]["p50"], d["cfg3"]["limit20"]["time_to_first_20_us"]["p50"],
          "shim", d["shim"]["query_us"]["p50"], d["shim"]["vs_batched"])
PY
fi
if has hostprof; then  # host phase times (TSG_PROF): the main line + limit-20, then the shim pattern alone
  TSG_PROF=1 timeout -k 10 300 python bench.py --steps 300 --cpu-baseline 0 --concurrent-steps 0 --cfg3 0 --cfg4 0 \
    --mall-steps 0 --shim-steps 0 > gpurun_out/hostprof_main.json 2> gpurun_out/hostprof_main.err
  rc=$?; echo "hostprof main rc=$rc"; tail -30 gpurun_out/hostprof_main.err
  [ $rc -eq 0 ] || exit $rc
  TSG_PROF=1 timeout -k 10 300 python bench.py --steps 20 --cpu-baseline 0 --concurrent-steps 0 --cfg3 0 --cfg4 0 \
    --mall-steps 0 --limit-steps 0 --shim-steps 300 > gpurun_out/hostprof_shim.json 2> gpurun_out/hostprof_shim.err
  rc=$?; echo "hostprof shim rc=$rc"; tail -30 gpurun_out/hostprof_shim.err
  [ $rc -eq 0 ] || exit $rc
fi
if has sweep; then  # pool-kernel knobs on the main line (blocks generated once, reused)
  W=/tmp/tsg_sweep; mkdir -p $W
  for cfg in "20 4" "30 4" "30 3" "40 3" "20 3"; do
    set -- $cfg
    TSG_POOL_DYN=$1 TSG_POOL_CHUNK=$2 timeout -k 10 300 python bench.py --steps 400 --cpu-baseline 0 --concurrent-steps 0 \
      --cfg3 0 --cfg4 0 --mall-steps 0 --shim-steps 0 --limit-steps 0 --workdir $W --events 2 > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err
    rc=$?; echo "sweep dyn=$1 chunk=$2 rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 -c "import json; d=json.load(open('gpurun_out/sweep_$1_$2.json')); print('  value', round(d['value']/1e9,1), 'frac', round(d['roofline']['frac'],3), 'kernel', d['latency_us']['kernel'])"
  done
fi
if has cfg4; then  # dictionary-stream parity, then the config-4 leg alone
  timeout -k 10 400 python -u -m pytest tests/test_gpu_dict_stream.py tests/test_gpu_configs.py -k "stream or cfg4" -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cfg4.log 2>&1
  rc=$?; echo "pytest cfg4 rc=$rc"; tail -2 gpurun_out/pytest_cfg4.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python bench.py --steps 20 --cpu-baseline 0 --concurrent-steps 0 --cfg3 0 --cfg4 1 --mall-steps 0 \
    --shim-steps 0 --limit-steps 0 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err
  rc=$?; echo "cfg4 bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/cfg4.json'))['cfg4']['queries']; [print(k, v['dict_pass_us']['p50'], round(v['dict_frac'],3), v['scan_us']['p50']) for k,v in d.items()]"
fi
if has cfg4prof; then  # per-kernel times of the config-4 leg
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --cpu-baseline 0 --concurrent-steps 0 --cfg3 0 --cfg4 1 --mall-steps 0 \
    --shim-steps 0 --limit-steps 0 > gpurun_out/c4prof.json 2> gpurun_out/c4prof.err
  rc=$?; echo "cfg4 rocprof rc=$rc"; head -12 gpurun_out/c4prof/run_kernel_stats.csv
  [ $rc -eq 0 ] || exit $rc
fi
if has sweep2; then
  W=/tmp/tsg_sweep; mkdir -p $W
  for cfg in "20 4" "30 4" "30 5" "40 4" "50 4" "30 4" "20 4"; do
    set -- $cfg
    TSG_POOL_DYN=$1 TSG_POOL_CHUNK=$2 timeout -k 10 300 python bench.py --steps 400 --cpu-baseline 0 --concurrent-steps 0 \
      --cfg3 0 --cfg4 0 --mall-steps 0 --shim-steps 0 --limit-steps 0 --workdir $W --events 4 > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err
    rc=$?; echo "sweep dyn=$1 chunk=$2 rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 -c "import json; d=json.load(open('gpurun_out/sweep_$1_$2.json')); print('  value', round(d['value']/1e9,1), 'frac', round(d['roofline']['frac'],3), 'kernel', d['latency_us']['kernel'])"
  done
fi
if has limprof; then  # the limit-20 leg alone under TSG_PROF: static-run vs pool kernel for the waves
  for su in 32 0; do
    TSG_PROF=1 TSG_POOL_STATIC_UNITS=$su timeout -k 10 300 python bench.py --steps 20 --cpu-baseline 0 --concurrent-steps 0 \
      --cfg3 0 --cfg4 0 --mall-steps 0 --shim-steps 0 --limit-steps 300 > gpurun_out/limprof_$su.json 2> gpurun_out/limprof_$su.err
    rc=$?; echo "limprof units=$su rc=$rc"; grep "prof p50" gpurun_out/limprof_$su.err
    [ $rc -eq 0 ] || exit $rc
    python3 -c "import json; d=json.load(open('gpurun_out/limprof_$su.json'))['limit20']; print(' step', d['step_us'], 'kernel', d['kernel_us']['p50'])"
  done
fi
if has mainstamps; then  # workgroup stamps of the main line's pool kernel only
  TSG_STAMPS=1 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-baseline 0 --cfg3 0 --cfg4 0 --concurrent-steps 0 \
    --mall-steps 0 --shim-steps 0 --limit-steps 0 > gpurun_out/mainstamps.json 2> gpurun_out/mainstamps.err
  rc=$?; echo "main stamps rc=$rc"; grep "stamps" gpurun_out/mainstamps.err | tail -6
  [ $rc -eq 0 ] || exit $rc
fi
if has quick; then
  timeout -k 10 600 python bench.py --steps 200 --cpu-baseline 0 --cfg3 0 --concurrent-steps 0 ${BENCH_ARGS:-} \
    > gpurun_out/quick.json 2> gpurun_out/quick.err
  rc=$?; echo "quick rc=$rc"; tail -2 gpurun_out/quick.err; cat gpurun_out/quick.json
  [ $rc -eq 0 ] || exit $rc
fi
if has driver; then  # the driver's own bench command
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver.json 2> gpurun_out/driver.err
  rc=$?; echo "driver bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/driver.json')); print('  value', round(d['value']/1e9,1), 'frac', round(d['roofline']['frac'],3), 'kernel', d['latency_us']['kernel'], 'step', d['latency_us']['step']['p50'])"
fi
if has bench; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 40 --warmup 3 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --concurrent-steps 0 --shim-steps 0 --cfg4 0 \
    --mall-steps 0 ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof/run_kernel_stats.csv
  [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --concurrent-steps 0 --shim-steps 0 --cfg4 0 \
      --mall-steps 0 ${BENCH_ARGS:-} > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
    rc=$?; echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE --out gpurun_out/pmc_traffic.json \
    --workload "${PMC_WORKLOAD:-blocks=10,entries=1000000,sets=4}" --source "${PMC_SOURCE:-tools/gpu_r3.sh pmc}" | tee gpurun_out/pmc_summary.txt
fi
exit 0
