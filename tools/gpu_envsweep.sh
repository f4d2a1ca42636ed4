#!/bin/bash
# Config-2 bench (HBM rotation) under env variants: value, step p50, kernel p50, roofline frac.
# usage: tools/gpu_envsweep.sh "default PER_CU=3 HIP_FORCE_DEV_KERNARG=1 ..."   (TSG_ prefix implied
# unless HIP_; a trailing @tag makes repeated names distinct)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in $1; do
  envs=()
  [ "${st%%@*}" != "default" ] && for kv in ${st//,/ }; do case $kv in HIP_*) envs+=("$kv");; *) envs+=("TSG_${kv%%@*}");; esac; done
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --cpu-baseline 0 --limit-steps 0 --cfg3 0 --concurrent-steps 0 \
    --mall-steps ${MALL:-0} --workdir /tmp/tsgw > gpurun_out/env_$st.json 2> gpurun_out/env_$st.err || { echo "$st failed"; tail -3 gpurun_out/env_$st.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('%-28s value %6.1f G/s  step p50 %5.1f us  kernel p50 %5.1f us  frac %.3f' % (sys.argv[2], d['value']/1e9,
      d['latency_us']['step']['p50'], d['latency_us']['kernel']['p50'], r['frac'] or 0))" gpurun_out/env_$st.json "$st"
done
