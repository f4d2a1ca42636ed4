#!/bin/bash
# Pool-path session: GPU tests (pool on, then off), stamps, host phases, bench A/B sweep.
# STAGES (comma list): test,testoff,stamps,prof,sweep. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${STAGES:-test,testoff,stamps,prof,sweep}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
B="python bench.py --cpu-baseline 0 --limit-steps 0 --mall-steps 0 --cfg3 0 --concurrent-steps 0 --workdir /tmp/tsgw"
if has test; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if has testoff; then
  TSG_NO_POOL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_nopool.log 2>&1
  rc=$?; echo "pytest gpu (TSG_NO_POOL) rc=$rc"; tail -2 gpurun_out/pytest_gpu_nopool.log; [ $rc -eq 0 ] || exit $rc
fi
if has stamps; then
  TSG_STAMPS=1 timeout -k 10 300 $B --steps 6 --warmup 2 > gpurun_out/st.json 2> gpurun_out/st.err
  rc=$?; grep stamps gpurun_out/st.err | tail -2; [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  for v in default NO_POOL; do
    if [ $v = default ]; then e=(); else e=("TSG_$v=1"); fi
    env "${e[@]}" TSG_PROF=1 timeout -k 10 300 $B --steps 200 --warmup 10 > gpurun_out/prof_$v.json 2> gpurun_out/prof_$v.err
    rc=$?; echo "$v: $(grep 'prof p50' gpurun_out/prof_$v.err | tail -1)"; [ $rc -eq 0 ] || exit $rc
  done
fi
if has sweep; then
  bash tools/gpu_envsweep.sh "${SWEEP:-default NO_POOL=1 default@2 NO_POOL=1@2}"
fi
