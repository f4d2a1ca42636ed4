#!/bin/bash
# Round-4 GPU session, second script: targeted tests, the config-4 leg, host phase profile of
# the main line (TSG_PROF=1). Stages by $1 (comma list); each GPU step under its own timeout,
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-tests,cfg4}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
if has tests; then
  timeout -k 10 500 $T -m gpu ${TESTS:-tests/test_gpu_dict_stream.py tests/test_gpu_block_filter.py tests/test_gpu_configs.py tests/test_gpu_coalesce.py} > gpurun_out/pt.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
if has cfg4; then
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --cfg3 0 --cfg5 0 --shim-steps 0 --limit-steps 0 \
    --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 > gpurun_out/b4.json 2> gpurun_out/b4.err
  rc=$?; echo "cfg4 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/b4.err; exit $rc; }
fi
if has hostprof; then
  TSG_PROF=1 timeout -k 10 500 python -u bench.py --steps 200 --warmup 20 --cfg3 0 --cfg4 0 --cfg5 0 --shim-steps 0 \
    --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/hp.json 2> gpurun_out/hp.err
  rc=$?; echo "hostprof rc=$rc"; grep -v "^\[bench\]" gpurun_out/hp.err | tail -40; [ $rc -eq 0 ] || exit $rc
fi
if has ab; then  # A/B of library builds on the main line: $AB_VARIANTS (dirs holding libtsg.so; "new" = the tree's), interleaved
  mkdir -p /tmp/abw
  for k in 1 2; do
    for v in ${AB_VARIANTS:-ab_old new}; do
      if [ $v = new ]; then unset TSG_LIB_PATH; else export TSG_LIB_PATH=$PWD/$v/libtsg.so; fi
      timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps ${AB_STEPS:-400} --warmup 20 --cfg3 0 --cfg4 0 --cfg5 0 \
        --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$k.json 2> gpurun_out/ab_${v}_$k.err
      rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; tail -3 gpurun_out/ab_${v}_$k.err; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); l=d['latency_us']; print(sys.argv[2], 'step mean %.1f p50 %.1f kernel mean %.2f' % (l['step']['mean'], l['step']['p50'], l['kernel']['mean']), 'lim20', round(d.get('limit20',{}).get('step_us',{}).get('mean',0),1))" gpurun_out/ab_${v}_$k.json $v
    done
  done
  unset TSG_LIB_PATH
fi
if has stamps; then  # workgroup stamps of the main-line kernel, per library variant
  mkdir -p /tmp/abw
  for v in ${AB_VARIANTS:-ab_old new}; do
    if [ $v = new ]; then unset TSG_LIB_PATH; else export TSG_LIB_PATH=$PWD/$v/libtsg.so; fi
    TSG_STAMPS=1 timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 16 --warmup 8 --cfg3 0 --cfg4 0 --cfg5 0 \
      --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --limit-steps 0 ${BENCH_ARGS:-} > gpurun_out/st_$v.json 2> gpurun_out/st_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "stamps $v rc=$rc"; tail -3 gpurun_out/st_$v.err; exit $rc; }
    echo "== $v"; grep "\[tsg\]" gpurun_out/st_$v.err | tail -6
  done
  unset TSG_LIB_PATH
fi
