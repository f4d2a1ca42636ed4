#!/bin/bash
# Round-5 GPU session script. Stages by $1 (comma list); each GPU step under its own timeout,
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${1:-tests,driver}"
has() { [[ ",$STAGES," == *",$1,"* ]]; }
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="--cfg3 0 --cfg4 0 --cfg5 0 --shim-steps 0 --concurrent-steps 0 --mall-steps 0 --cpu-baseline 0 --parity 0"
summ() {  # one-line summary of a bench JSON line
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = d.get("latency_us", {})
out = [sys.argv[2], "value %.1fG" % (d["value"] / 1e9), "frac %s" % (round(d["roofline"]["frac"], 3) if d["roofline"]["frac"] else None),
       "step mean %.1f p50 %.1f" % (l["step"]["mean"], l["step"]["p50"]) if l.get("step") else "",
       "kernel mean %.2f" % l["kernel"]["mean"] if l.get("kernel") else ""]
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
if has over; then  # the oversubscribed shim test, host phases on (non-fatal: the stages after it still run)
  TSG_PROF=1 timeout -k 10 300 $T -m gpu tests/test_gpu_coalesce.py -k oversubscribed > gpurun_out/over.log 2>&1
  echo "over rc=$?"; grep -E "slowest|passed|failed" gpurun_out/over.log | tail -3; grep -o "coal.park[a-z_]*=[^ ]*" gpurun_out/over.log | head -8
fi
if has tests; then
  timeout -k 10 600 $T -m gpu ${TESTS:-tests/test_gpu_coalesce.py tests/test_gpu_pool.py --deselect tests/test_gpu_coalesce.py::test_shim_limit20_oversubscribed} > gpurun_out/pt.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
if has alltests; then
  timeout -k 10 900 $T -m gpu tests > gpurun_out/pt_all.log 2>&1
  rc=$?; echo "alltests rc=$rc"; tail -4 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
fi
if has driver; then  # the driver's own command
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver.json 2> gpurun_out/driver.err
  rc=$?; echo "driver rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/driver.err; exit $rc; }
  summ gpurun_out/driver.json driver
fi
if has resab; then  # resident kernel on/off, interleaved (main line + limit 20)
  mkdir -p /tmp/abw
  for k in 1 2; do
    for m in 1 0; do
      TSG_RESIDENT=$m timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 400 --warmup 20 $B ${BENCH_ARGS:-} \
        > gpurun_out/res_${m}_$k.json 2> gpurun_out/res_${m}_$k.err
      rc=$?; [ $rc -eq 0 ] || { echo "resab $m rc=$rc"; tail -3 gpurun_out/res_${m}_$k.err; exit $rc; }
      summ gpurun_out/res_${m}_$k.json "resident=$m"
    done
  done
fi
if has share2; then  # the N=2 legs on one GPU (ranks share device 0, gloo)
  timeout -k 10 900 python3 bench.py --gpus 2 --ranks-share-gpu --steps 20 --warmup 5 > gpurun_out/share2.json 2> gpurun_out/share2.err
  rc=$?; echo "share2 rc=$rc"; [ $rc -eq 0 ] || { tail -8 gpurun_out/share2.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/share2.json').read().strip().splitlines()[-1]); print({k: (d[k] if not isinstance(d[k], dict) else sorted(d[k].keys())) for k in ('n_gpus','value','merge','cfg3','cfg5','parity_all_ranks') if k in d})"
fi
if has shim; then  # the shim leg alone, a few times
  for k in 1 2 3; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cfg3 0 --cfg4 0 --cfg5 0 --concurrent-steps 0 \
      --mall-steps 0 --cpu-baseline 0 --parity 0 --limit-steps 0 --shim-steps 400 > gpurun_out/shim_$k.json 2> gpurun_out/shim_$k.err
    rc=$?; [ $rc -eq 0 ] || { echo "shim rc=$rc"; tail -3 gpurun_out/shim_$k.err; exit $rc; }
    summ gpurun_out/shim_$k.json shim$k
  done
fi
if has fence; then  # AQL argument-visibility modes, interleaved
  mkdir -p /tmp/abw
  for k in 1 2; do
    for m in hdp sfence readback; do
      TSG_AQL_FENCE=$m timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 400 --warmup 20 $B ${BENCH_ARGS:-} \
        > gpurun_out/fence_${m}_$k.json 2> gpurun_out/fence_${m}_$k.err
      rc=$?; [ $rc -eq 0 ] || { echo "fence $m rc=$rc"; tail -3 gpurun_out/fence_${m}_$k.err; exit $rc; }
      summ gpurun_out/fence_${m}_$k.json "fence-$m"
    done
  done
fi
if has hostprof; then
  TSG_PROF=1 timeout -k 10 500 python -u bench.py --steps 200 --warmup 20 $B ${BENCH_ARGS:-} > gpurun_out/hp.json 2> gpurun_out/hp.err
  rc=$?; echo "hostprof rc=$rc"; grep -v "^\[bench\]" gpurun_out/hp.err | tail -4; [ $rc -eq 0 ] || exit $rc
fi
if has resprof; then  # host phases + workgroup stamp spread, resident on and off
  for m in 1 0; do
    TSG_PROF=1 TSG_RES_DUMP=1 TSG_RESIDENT=$m timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 $B --limit-steps 0 \
      > gpurun_out/rp_$m.json 2> gpurun_out/rp_$m.err
    rc=$?; echo "resprof $m rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/rp_$m.err; exit $rc; }
    summ gpurun_out/rp_$m.json "prof resident=$m"
    grep "resident stamps" gpurun_out/rp_$m.err | tail -3
    grep -o "plan=[0-9.]*\|search=[0-9.]*\|sync=[0-9.]*\|post=[0-9.]*\|post.keys=[0-9.]*\|post.sort=[0-9.]*\|res.first_count=[0-9.]*\|tsg_search.results=[0-9.]*\|tsg_search.device=[0-9.]*" gpurun_out/rp_$m.err | tr '\n' ' '; echo
  done
fi
if has resvar; then  # resident kernel variants (TSG_RES_MODE bits, TSG_RES_PREFETCH), host phases each
  for v in "TSG_RES_MODE=0" "TSG_RES_MODE=1" "TSG_RES_MODE=2" "TSG_RES_PREFETCH=0" "TSG_RESIDENT=0"; do
    env $v TSG_PROF=1 timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 200 --warmup 20 $B --limit-steps 0 \
      > gpurun_out/rv.json 2> gpurun_out/rv.err
    rc=$?; [ $rc -eq 0 ] || { echo "resvar $v rc=$rc"; tail -3 gpurun_out/rv.err; exit $rc; }
    summ gpurun_out/rv.json "$v"
    grep -o "res.first_count=[0-9.]*\|sync=[0-9.]*\|post=[0-9.]*" gpurun_out/rv.err | head -3 | tr '\n' ' '; echo
  done
fi
if has resdiag; then  # every query timed: the span per query, by resident set
  for a in "--sets 4 --events 1" "--sets 1 --events 1" "--sets 4 --events 4"; do
    TSG_RES_DUMP=1 TSG_PROF=1 timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 40 --warmup 8 $B --limit-steps 0 $a \
      > gpurun_out/rd.json 2> gpurun_out/rd.err
    rc=$?; [ $rc -eq 0 ] || { echo "resdiag rc=$rc"; tail -3 gpurun_out/rd.err; exit $rc; }
    summ gpurun_out/rd.json "$a"
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/rd.json').read().strip().splitlines()[-1])
print('kernel_us', [round(x) for x in d['latency_us']['kernel'].values()])
"
    grep "resident stamps" gpurun_out/rd.err | awk '{print \$NF}' | tail -24 | tr '\n' ' '; echo
  done
fi
if has c45prof; then  # configs 4 and 5 with host phases; look-back records compact vs full
  for v in ${C45_VARIANTS:-TSG_PROF=1 TSG_LB_FULL=1}; do  # (variants: env assignments, run in order)
    env $v TSG_PROF=1 timeout -k 10 400 python -u tools/c45_prof.py --parity 0 ${BENCH_ARGS:-} \
      > gpurun_out/c45_$v.json 2> gpurun_out/c45_$v.err
    rc=$?; echo "c45prof $v rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/c45_$v.err; exit $rc; }
    python3 tools/prof_table.py gpurun_out/c45_$v.err sync post tsg_search.results.records fill.names fill.records tsg_search.results.finalize tsg_search.device
    python3 -c "
import json
d=json.loads(open('gpurun_out/c45_$v.json').read().strip().splitlines()[-1])
for n,q in d['cfg4']['queries'].items(): print(n, 'step', round(q['step_us']['p50']), 'dev', round(q['device_us']['p50']), 'scan', round(q['scan_us']['p50']), 'dict', round(q['dict_pass_us']['p50']), 'matches', q['matches'])
c=d['cfg5']; print('cfg5 dev_ms', c['device_ms'], 'host_e2e p50', round(c['host_e2e']['step_ms']['p50'],2))
"
  done
fi
if has varab; then  # env variants of the main line, interleaved twice (VARS: space-separated env assignments; "-" = none)
  mkdir -p /tmp/abw
  for k in 1 2; do
    for v in ${VARS:--}; do
      e="$v"; [ "$v" = "-" ] && e="TSG_NONE=1"
      env $e TSG_PROF=1 timeout -k 10 300 python -u bench.py --workdir /tmp/abw --steps 400 --warmup 20 $B --limit-steps 0 --cfg1 0 \
        > gpurun_out/var.json 2> gpurun_out/var.err
      rc=$?; [ $rc -eq 0 ] || { echo "varab $v rc=$rc"; tail -3 gpurun_out/var.err; exit $rc; }
      summ gpurun_out/var.json "$v"
      grep "prof p50" gpurun_out/var.err | tail -1 | tr ' ' '\n' | grep -E "^(res.first_count|sync|tsg_search.device|tsg_search.results)=" | tr '\n' ' '; echo
    done
  done
fi
if has pmc; then  # FETCH_SIZE / WRITE_SIZE passes of the main line as plain launches (per-dispatch counters)
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    TSG_RESIDENT=0 timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 $B --limit-steps 0 --cfg1 0 > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
    rc=$?; echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE --out gpurun_out/pmc_traffic.json \
    --workload "${PMC_WORKLOAD:-blocks=10,entries=1000000,sets=4,layout=ds}" --source "${PMC_SOURCE:-gpu_r5.sh pmc}" | tee gpurun_out/pmc_summary.txt
fi
if has smoke; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if has stamps; then  # resident spans per workgroup on the main line (TSG_RES_DUMP), host phases
  TSG_RES_DUMP=1 TSG_PROF=1 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 $B --cfg1 0 --limit-steps 0 \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err
  rc=$?; echo "stamps rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep "resident stamps" gpurun_out/stamps.err | tail -3
fi
if has rocprof; then  # kernel trace + stats of the main line (profiles/)
  cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
  TSG_RESIDENT=${ROCPROF_RESIDENT:-0} timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp -o rp -- python3 bench.py --steps 200 --warmup 10 $B --cfg1 0 \
    > gpurun_out/rp.json 2> gpurun_out/rp.err
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/rp.err; exit $rc; }
  find gpurun_out/rp -name "*kernel_stats.csv" | head -3
fi
echo "done: $STAGES"
