#!/bin/bash
# Host-side step breakdown (TSG_PROF medians) of the config-2 search under env settings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in ${1:-"ev0 ev1 MARK=1 MARK=2 MARK=3"}; do
  envs=(TSG_PROF=1); ev=0
  case $st in ev1) ev=1 ;; ev0) ;; *) for kv in ${st//,/ }; do envs+=("TSG_$kv"); done ;; esac
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-400} --warmup 10 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --concurrent-steps 0 --mall-steps 0 \
    --events $ev --workdir /tmp/tsgw > gpurun_out/host_$st.json 2> gpurun_out/host_$st.err || { echo "$st failed"; tail -3 gpurun_out/host_$st.err; exit 1; }
  echo "== $st: $(grep 'prof p50' gpurun_out/host_$st.err | cut -c18-)"
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('   step', {k: round(v,1) for k,v in d['latency_us']['step'].items()}, 'value %.1f G/s' % (d['value']/1e9))" gpurun_out/host_$st.json
done
