#!/bin/bash
# (1) main + shim legs with TSG_PROF (where a slow limit-20 shim query spends its time);
# (2) rocprofv3 kernel trace of the config-4 leg alone (dictionary-pass kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TSG_PROF=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --mall-steps 0 --limit-steps 0 --cfg3 0 --cfg4 0 --cfg5 0 \
  --concurrent-steps 0 --parity 0 --cpu-baseline 0 --shim-steps 400 > gpurun_out/shimprof.json 2> gpurun_out/shimprof.err
rc=$?; echo "shimprof rc=$rc"; grep "prof" gpurun_out/shimprof.err; python3 -c "
import json; d=json.load(open('gpurun_out/shimprof.json')); print(d['shim'])"
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg4 -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --mall-steps 0 --limit-steps 0 --shim-steps 0 --concurrent-steps 0 --cfg3 0 --cfg5 0 \
  --parity 0 --cpu-baseline 0 --cfg4-steps 5 > gpurun_out/prof_cfg4.json 2> gpurun_out/prof_cfg4.err
rc=$?; echo "rocprof cfg4 rc=$rc"; cat gpurun_out/prof_cfg4/run_kernel_stats.csv | cut -c1-250
exit $rc
