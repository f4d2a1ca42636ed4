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
if has wave0; then  # the limit-20 legs at several first-wave sizes (TSG_LIMIT_WAVE0)
  mkdir -p /tmp/abw
  for wz in ${WAVE0S:-2097152 1048576 524288}; do
    TSG_LIMIT_WAVE0=$wz timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 50 --warmup 10 --cfg4 0 --cfg5 0 \
      --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --limit-steps 200 ${BENCH_ARGS:-} > gpurun_out/w0_$wz.json 2> gpurun_out/w0_$wz.err
    rc=$?; [ $rc -eq 0 ] || { echo "wave0 $wz rc=$rc"; tail -3 gpurun_out/w0_$wz.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); l=d['limit20']; c=d.get('cfg3',{}).get('limit20',{}); print('wave0', sys.argv[2], 'lim20 step mean %.1f p50 %.1f kernel mean %.2f' % (l['step_us']['mean'], l['step_us']['p50'], l['kernel_us']['mean']), 'cfg3 first20 p50 %.1f mean %.1f' % (c.get('time_to_first_20_us',{}).get('p50',0), c.get('time_to_first_20_us',{}).get('mean',0)))" gpurun_out/w0_$wz.json $wz
  done
fi
if has limstamps; then  # workgroup stamps of the limit-20 first wave (static kernel)
  mkdir -p /tmp/abw
  TSG_STAMPS=1 timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 2 --warmup 1 --cfg3 0 --cfg4 0 --cfg5 0 \
    --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --limit-steps 12 ${BENCH_ARGS:-} > gpurun_out/ls.json 2> gpurun_out/ls.err
  rc=$?; [ $rc -eq 0 ] || { echo "limstamps rc=$rc"; tail -3 gpurun_out/ls.err; exit $rc; }
  grep "\[tsg\]" gpurun_out/ls.err | tail -8
fi
if has cfg4prof; then  # host phases of the config-4 leg (TSG_PROF)
  mkdir -p /tmp/abw
  TSG_PROF=1 timeout -k 10 400 python -u bench.py --workdir /tmp/abw --steps 3 --warmup 1 --cfg3 0 --cfg5 0 --shim-steps 0 \
    --limit-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --cfg4-steps 10 > gpurun_out/c4p.json 2> gpurun_out/c4p.err
  rc=$?; echo "cfg4prof rc=$rc"; grep -v "^\[bench\]" gpurun_out/c4p.err | tail -6; [ $rc -eq 0 ] || exit $rc
fi
if has abcfg4; then  # A/B of library builds on the config-4 leg, interleaved
  mkdir -p /tmp/abw
  for k in 1 2; do
    for v in ${AB_VARIANTS:-ab_old new}; do
      if [ $v = new ]; then unset TSG_LIB_PATH; else export TSG_LIB_PATH=$PWD/$v/libtsg.so; fi
      timeout -k 10 400 python -u bench.py --workdir /tmp/abw --steps 3 --warmup 1 --cfg3 0 --cfg5 0 --shim-steps 0 --limit-steps 0 \
        --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --cfg4-steps 10 > gpurun_out/a4_${v}_$k.json 2> gpurun_out/a4_${v}_$k.err
      rc=$?; [ $rc -eq 0 ] || { echo "abcfg4 $v rc=$rc"; tail -3 gpurun_out/a4_${v}_$k.err; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); q=d['cfg4']['queries']; print(sys.argv[2], ' '.join('%s %.0f/%.3f' % (n[:9], v['dict_pass_us']['p50'], v['dict_frac']) for n, v in q.items()))" gpurun_out/a4_${v}_$k.json $v
    done
  done
  unset TSG_LIB_PATH
fi
