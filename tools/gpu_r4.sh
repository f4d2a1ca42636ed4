#!/bin/bash
# Round-4 GPU-box session: stages chosen by $1 (comma list). Every GPU step runs under its
# own timeout; the script stops at the first failure (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-new,gputest}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 test failures (no crash)
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"

if has new; then  # this round's new / changed GPU tests first
  timeout -k 10 600 $T -m gpu tests/test_gpu_limit_ranks.py tests/test_gpu_block_filter.py tests/test_gpu_coalesce.py tests/test_gpu_multiproc.py \
    tests/test_gpu_configs.py > gpurun_out/pytest_new.log 2>&1
  rc=$?; echo "pytest new rc=$rc"; tail -25 gpurun_out/pytest_new.log
  [ $rc -eq 0 ] || exit $rc
fi
if has gputest; then
  timeout -k 10 900 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -12 gpurun_out/bench.err; cut -c1-3000 gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if has driver; then  # the driver's own command
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver.json 2> gpurun_out/driver.err
  rc=$?; echo "driver bench rc=$rc"; tail -12 gpurun_out/driver.err; cut -c1-3000 gpurun_out/driver.json
  [ $rc -eq 0 ] || exit $rc
fi
if has gpus2; then  # the launcher on a 1-GPU box: must refuse with a clear message
  timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/gpus2.out 2> gpurun_out/gpus2.err
  rc=$?; echo "bench --gpus 2 rc=$rc (expected 2)"; tail -2 gpurun_out/gpus2.err
  [ $rc -eq 2 ] || exit 1
fi
if has prof; then
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --cfg4 0 --cfg5 0 --shim-steps 0 \
    --concurrent-steps 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?; echo "rocprof rc=$rc"; head -12 gpurun_out/prof/run_kernel_stats.csv
  [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --cfg4 0 --cfg5 0 --shim-steps 0 \
      --concurrent-steps 0 --mall-steps 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
    rc=$?; echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE --out gpurun_out/pmc_traffic.json \
    --workload "${PMC_WORKLOAD:-blocks=10,entries=1000000,sets=4,layout=ds}" --source "${PMC_SOURCE:-gpu_r4.sh pmc}" | tee gpurun_out/pmc_summary.txt
fi
