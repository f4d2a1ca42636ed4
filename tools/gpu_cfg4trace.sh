#!/bin/bash
# config-4 leg alone with per-search host phase traces (TSG_TRACE): where a dense query's host time goes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TSG_TRACE=1 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --mall-steps 0 --limit-steps 0 --shim-steps 0 \
  --concurrent-steps 0 --cfg3 0 --cfg5 0 --parity 0 --cpu-baseline 0 --cfg4-steps 4 > gpurun_out/cfg4trace.json 2> gpurun_out/cfg4trace.err
rc=$?; echo "rc=$rc"; grep "\[tsg\]" gpurun_out/cfg4trace.err | tail -40; exit $rc
