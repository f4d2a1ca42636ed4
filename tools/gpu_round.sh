#!/bin/bash
# One GPU-box session: tests, bench, rocprof. Stops at the first GPU fault/abort/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-test,bench,prof}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 test failures (no crash)

if has test; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  ok_rc $rc || exit $rc
  # narrow full scans on the one-launch segment kernel instead of the pool kernel
  TSG_NO_POOL=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_nopool.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_POOL) rc=$rc"; tail -5 gpurun_out/pytest_gpu_nopool.log
  ok_rc $rc || exit $rc
  # the general (prep kernel + descriptor) search path, forced
  TSG_NO_FAST=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_nofast.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_FAST) rc=$rc"; tail -5 gpurun_out/pytest_gpu_nofast.log
  ok_rc $rc || exit $rc
  # the one-launch path with dictionary workgroups (granule hand-off) instead of per-workgroup matching
  TSG_NO_NARROW=1 TSG_NO_SELF_DICT=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_noself.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_SELF_DICT) rc=$rc"; tail -5 gpurun_out/pytest_gpu_noself.log
  ok_rc $rc || exit $rc
  # the one-launch path without host-matched narrow dictionaries (self-matching workgroups)
  TSG_NO_NARROW=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py tests/test_gpu_wal.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_nonarrow.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_NARROW) rc=$rc"; tail -5 gpurun_out/pytest_gpu_nonarrow.log
  ok_rc $rc || exit $rc
  # segment mode without tail work stealing (static tile split only)
  TSG_STEAL=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_steal.log 2>&1
  rc=$?; echo "pytest gpu (TSG_STEAL) rc=$rc"; tail -5 gpurun_out/pytest_gpu_steal.log
  ok_rc $rc || exit $rc
  # one descriptor-path launch for blocks beyond 32 (no chunking)
  TSG_CHUNK_BLOCKS=0 timeout -k 10 600 python -m pytest tests/test_gpu_search.py -m gpu -x -q -p no:cacheprovider -k "many_blocks or cancel or limit" > gpurun_out/pytest_gpu_nochunk.log 2>&1
  rc=$?; echo "pytest gpu (TSG_CHUNK_BLOCKS=0) rc=$rc"; tail -5 gpurun_out/pytest_gpu_nochunk.log
  ok_rc $rc || exit $rc
  # the one-launch path in look-back mode only (no per-tile segments)
  TSG_NO_SEG=1 timeout -k 10 600 python -m pytest tests/test_gpu_search.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_noseg.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_SEG) rc=$rc"; tail -5 gpurun_out/pytest_gpu_noseg.log
  ok_rc $rc || exit $rc
fi
if has trace; then
  TSG_TRACE=1 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/trace.json 2> gpurun_out/trace.err
  rc=$?; echo "trace rc=$rc"; grep "\[tsg\]" gpurun_out/trace.err | tail -6; cat gpurun_out/trace.json
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 --events 0 ${BENCH_ARGS:-} > gpurun_out/noevents.json 2> gpurun_out/noevents.err
  rc=$?; echo "noevents rc=$rc"; cat gpurun_out/noevents.json
  [ $rc -eq 0 ] || exit $rc
  TSG_EXT_EVENTS=1 timeout -k 10 600 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/extevents.json 2> gpurun_out/extevents.err
  rc=$?; echo "extevents rc=$rc"; cat gpurun_out/extevents.json
  [ $rc -eq 0 ] || exit $rc
fi
if has stamps; then
  TSG_STAMPS=1 TSG_TRACE=1 timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/stamps.json 2> gpurun_out/stamps.err
  rc=$?; echo "stamps rc=$rc"; grep "stamps" gpurun_out/stamps.err | tail -3
  [ $rc -eq 0 ] || exit $rc
  TSG_NO_FAST=1 TSG_STAMPS=1 TSG_TRACE=1 timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/stamps_nofast.json 2> gpurun_out/stamps_nofast.err
  rc=$?; echo "stamps nofast rc=$rc"; grep "stamps\|tsg_search\|device_search" gpurun_out/stamps_nofast.err | tail -4
  [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if has lookup; then
  timeout -k 10 600 python tools/bench_lookup.py ${LOOKUP_ARGS:-} > gpurun_out/lookup.json 2> gpurun_out/lookup.err
  rc=$?; echo "lookup rc=$rc"; tail -3 gpurun_out/lookup.err; cat gpurun_out/lookup.json
  [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 --limit-steps 0 ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof/run_kernel_stats.csv
fi
if has pmc; then
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 900 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --limit-steps 0 ${BENCH_ARGS:-} > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
    rc=$?; echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE --out gpurun_out/pmc_traffic.json \
    --workload "${PMC_WORKLOAD:-blocks=10,entries=1000000}" --source "${PMC_SOURCE:-gpu_round.sh pmc}" | tee gpurun_out/pmc_summary.txt
fi

