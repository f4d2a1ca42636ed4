#!/bin/bash
# Lookup path on the GPU box: parity tests (slab and direct probing), the config-5 bench
# line, and its rocprofv3 kernel summary. Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_lookup.py tests/test_gpu_configs.py -k "lookup or find or cfg5 or fixture or blocks or range or devices" \
  > gpurun_out/lk_slab.log 2>&1 || { echo "slab tests failed"; tail -15 gpurun_out/lk_slab.log; exit 1; }
tail -1 gpurun_out/lk_slab.log
TSG_LK_SLAB=0 timeout -k 10 300 $T tests/test_gpu_lookup.py -k "synthetic or many or range or devices" \
  > gpurun_out/lk_direct.log 2>&1 || { echo "direct tests failed"; tail -15 gpurun_out/lk_direct.log; exit 1; }
tail -1 gpurun_out/lk_direct.log
TSG_LK_SLAB=1 timeout -k 10 300 $T tests/test_gpu_lookup.py -k "fixture or synthetic or many or range or devices" \
  > gpurun_out/lk_forced.log 2>&1 || { echo "forced-slab tests failed"; tail -15 gpurun_out/lk_forced.log; exit 1; }
tail -1 gpurun_out/lk_forced.log
timeout -k 10 600 python tools/bench_lookup.py ${LK_ARGS:-} > gpurun_out/lookup_bench.json 2> gpurun_out/lookup_bench.err \
  || { echo "bench_lookup failed"; tail -5 gpurun_out/lookup_bench.err; exit 1; }
cat gpurun_out/lookup_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof -o run --output-format csv -- \
  python3 tools/bench_lookup.py --cpu-sample 0 --check 2000 --steps 3 > gpurun_out/lkprof.json 2> gpurun_out/lkprof.err \
  || { echo "rocprof failed"; tail -5 gpurun_out/lkprof.err; exit 1; }
find gpurun_out/lkprof -name "*kernel_stats.csv" | head -1 | xargs cat
