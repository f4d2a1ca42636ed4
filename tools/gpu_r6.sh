#!/bin/bash
# Round-6 GPU session script. Stages by $1 (comma list); each GPU step under its own timeout,
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-new,quick}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="--cfg3 0 --cfg4 0 --cfg5 0 --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0 --cfg1 0"
summ() {  # one-line summary of a bench JSON line
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = d.get("latency_us", {})
out = [sys.argv[2], "value %.1fG" % (d["value"] / 1e9), "frac %s" % (round(d["roofline"]["frac"], 3) if d["roofline"]["frac"] else None),
       "step mean %.1f p50 %.1f" % (l["step"]["mean"], l["step"]["p50"]) if l.get("step") else "",
       "kernel mean %.2f" % l["kernel"]["mean"] if l.get("kernel") else ""]
if "batched" in d:
    b = d["batched"]
    out.append("batched dev/q %s wall/q %.1f frac %s ok %s" % (b["device_us_per_query"] and round(b["device_us_per_query"], 2),
                                                            b["wall_us_per_query"], b["frac"] and round(b["frac"], 3),
                                                            b["counts_match_and_resident"]))
if "limit20" in d:
    out.append("lim20 step mean %.1f" % d["limit20"]["step_us"]["mean"])
if "shim" in d:
    s = d["shim"]
    out.append("shim p50 %.1f p99 %.1f | lim20 p50 %.1f p99 %.1f max %.1f" % (
        s["query_us"]["p50"], s["query_us"]["p99"], s["limit20"]["query_us"]["p50"], s["limit20"]["query_us"]["p99"],
        s["limit20"]["query_us"]["max"]))
print(" ".join(out))
EOF
}
if has new; then
  timeout -k 10 600 $T -m gpu tests/test_gpu_resident2.py tests/test_gpu_multidevice.py tests/test_gpu_resident.py > gpurun_out/pt_new.log 2>&1
  rc=$?; echo "new rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pt_new.log | tail -30; tail -4 gpurun_out/pt_new.log; [ $rc -eq 0 ] || exit $rc
fi
if has mdev; then  # (non-fatal: the stages after it still run)
  TSG_SEGV_TRACE=1 timeout -k 10 400 $T -m gpu tests/test_gpu_multidevice.py > gpurun_out/pt_mdev.log 2>&1
  echo "mdev rc=$?"; grep -E "PASS|FAIL|Error|error|tsg\]|libtsg" gpurun_out/pt_mdev.log | head -60; tail -4 gpurun_out/pt_mdev.log
fi
if has cfg4; then
  timeout -k 10 600 $T -m gpu tests/test_gpu_dict_stream.py tests/test_gpu_block_filter.py tests/test_gpu_pipelined.py > gpurun_out/pt_cfg4.log 2>&1
  rc=$?; echo "cfg4 tests rc=$rc"; grep -E "FAIL|Error" gpurun_out/pt_cfg4.log | head -20; tail -3 gpurun_out/pt_cfg4.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --limit-steps 0 --batch-queries 0 --cfg3 0 --cfg5 0 --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --cfg1 0 --cfg4 1 --parity 1 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err
  rc=$?; echo "cfg4 bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/cfg4.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cfg4.json').read().strip().splitlines()[-1]); c=d['cfg4']
print('parity', c.get('parity',{}).get('ok'))
for k,v in c['queries'].items(): print(k, 'matches', v['matches'], 'scan_us', v['scan_us'], 'step_us p50/p99', v['step_us']['p50'], v['step_us']['p99'], 'dev p50', v['device_us']['p50'], 'sod', round(v['step_over_device'] or 0,2))
"
fi
if has cfg4ab; then  # pipelined chunk size A/B (TSG_PIPE_BLOCKS)
  for pb in 2 4; do
    TSG_PIPE_BLOCKS=$pb timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --limit-steps 0 --batch-queries 0 --cfg3 0 --cfg5 0 --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --cfg1 0 --cfg4 1 --cfg4-steps 20 --parity 0 > gpurun_out/cfg4_pb$pb.json 2> gpurun_out/cfg4_pb$pb.err
    rc=$?; echo "cfg4 pb=$pb rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/cfg4_pb$pb.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/cfg4_pb$pb.json').read().strip().splitlines()[-1]); c=d['cfg4']
for k,v in c['queries'].items(): print(' ', k, 'scan p50', v['scan_us']['p50'], 'step p50/p99 %.0f %.0f' % (v['step_us']['p50'], v['step_us']['p99']), 'dev p50 %.0f' % v['device_us']['p50'], 'sod %.2f' % (v['step_over_device'] or 0))
"
  done
fi
if has share2; then  # the N=2 path with both ranks on the one GPU (merged query: gloo and shared memory)
  timeout -k 10 600 python3 bench.py --gpus 2 --ranks-share-gpu --steps 100 --warmup 5 --merge-steps 50 $B --batch-queries 0 --limit-steps 0 > gpurun_out/share2.json 2> gpurun_out/share2.err
  rc=$?; echo "share2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/share2.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/share2.json').read().strip().splitlines()[-1]); m=d.get('merge',{})
print('value %.1fG step mean %.1f' % (d['value']/1e9, d['latency_us']['step']['mean']))
print('gloo merged step', m.get('step_us')); print('shm', m.get('shm'))
"
fi
if has rprof; then  # rocprofv3 over resident launches that each serve 64 batched queries
  RB="python3 bench.py --steps 8 --warmup 2 --limit-steps 0 --batch-queries 64 --batch-reps 6 $B"
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_res -o res -- $RB > gpurun_out/rp_res.json 2> gpurun_out/rp_res.err
  rc=$?; echo "rprof trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rp_res.err; exit $rc; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/rp_$c -o p -- $RB > gpurun_out/rp_$c.json 2> gpurun_out/rp_$c.err
    rc=$?; echo "rprof $c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rp_$c.err; exit $rc; }
  done
  find gpurun_out/rp_res gpurun_out/rp_FETCH_SIZE gpurun_out/rp_WRITE_SIZE -name "*.csv" | head -20
  summ gpurun_out/rp_res.json rp_res
fi
if has ab; then  # library builds side by side (AB="w8 w12": tools/_bin/<v>/libtsg.so + its code object)
  for v in ${AB:-w8 w12}; do
    L=$PWD/tools/_bin/$v/libtsg.so
    TSG_LIB_PATH=$L timeout -k 10 500 $T -m gpu ${ABTESTS:-tests/test_gpu_resident.py tests/test_gpu_pool.py} > gpurun_out/pt_ab_$v.log 2>&1
    rc=$?; echo "ab $v tests rc=$rc"; tail -n 2 gpurun_out/pt_ab_$v.log; [ $rc -eq 0 ] || exit $rc
    TSG_LIB_PATH=$L timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 $B > gpurun_out/quick_$v.json 2> gpurun_out/quick_$v.err
    rc=$?; echo "ab $v quick rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/quick_$v.err; exit $rc; }
    summ gpurun_out/quick_$v.json quick_$v
    TSG_LIB_PATH=$L TSG_RES_DUMP=1 timeout -k 10 400 python3 bench.py --steps 100 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/dump_$v.json 2> gpurun_out/dump_$v.err
    echo "ab $v dump rc=$?"; grep "resident stamps" gpurun_out/dump_$v.err | tail -3
  done
fi
if has tests; then
  timeout -k 10 600 $T -m gpu ${TESTS:-tests/test_gpu_coalesce.py tests/test_gpu_pool.py tests/test_gpu_search.py} > gpurun_out/pt.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
if has alltests; then
  timeout -k 10 900 $T -m gpu tests > gpurun_out/pt_all.log 2>&1
  rc=$?; echo "alltests rc=$rc"; tail -4 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
fi
if has quick; then
  timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 $B > gpurun_out/quick.json 2> gpurun_out/quick.err
  rc=$?; echo "quick rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/quick.err; exit $rc; }
  summ gpurun_out/quick.json quick
  TSG_RES_XSPLIT=0 timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/quick_nox.json 2> gpurun_out/quick_nox.err
  rc=$?; echo "quick_nox rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/quick_nox.err; exit $rc; }
  summ gpurun_out/quick_nox.json quick_noxsplit
fi
if has dump; then  # per-workgroup seen / end stamps of the timed main-line queries, XCD split on and off
  TSG_RES_DUMP=2 timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/dump_x.json 2> gpurun_out/dump_x.err
  echo "dump_x rc=$?"; summ gpurun_out/dump_x.json dump_x
  TSG_RES_XSPLIT=0 TSG_RES_DUMP=2 timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/dump_n.json 2> gpurun_out/dump_n.err
  echo "dump_n rc=$?"; summ gpurun_out/dump_n.json dump_n
fi
if has modes; then  # per-workgroup stamps under TSG_RES_MODE experiments (MODES="0 8 16")
  for m in ${MODES:-0 8 16}; do
    TSG_RES_MODE=$m TSG_RES_DUMP=2 timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/mode_$m.json 2> gpurun_out/mode_$m.err
    echo "mode $m rc=$?"; summ gpurun_out/mode_$m.json mode_$m
  done
fi
if has prof; then  # host phases of the main line
  TSG_PROF=1 timeout -k 10 400 python3 bench.py --steps 400 --warmup 5 --limit-steps 0 --batch-queries 0 $B > gpurun_out/prof.json 2> gpurun_out/prof.err
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof.err; exit $rc; }
  summ gpurun_out/prof.json prof; grep -E "^\[tsg\] prof|tsg_search|res\.|launch|sync|post" gpurun_out/prof.err | tail -40
fi
if has driver; then
  timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver.json 2> gpurun_out/driver.err
  rc=$?; echo "driver rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/driver.err; exit $rc; }
  summ gpurun_out/driver.json driver
fi
echo "all stages done"
