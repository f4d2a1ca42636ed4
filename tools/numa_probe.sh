#!/bin/bash
# Host placement probe: config-2 step time with the process on its GPU's NUMA node
# (bench.py --pin auto) vs on each node's CPUs (taskset, --pin none).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, launcher...
  local name=$1; shift
  timeout -k 10 300 "$@" python bench.py --steps 400 --warmup 10 --cpu-baseline 0 --limit-steps 0 --workdir /tmp/tsgw \
    ${PIN:-} > gpurun_out/numa_$name.json 2> gpurun_out/numa_$name.err || { tail -3 gpurun_out/numa_$name.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'step', {k: round(v,1) for k,v in d['latency_us']['step'].items()}, 'kernel p50 %.1f' % d['latency_us']['kernel']['p50'], 'value %.1f G/s' % (d['value']/1e9))" gpurun_out/numa_$name.json $name
  grep "NUMA" gpurun_out/numa_$name.err || true
}
run auto
PIN="--pin none" run node0 taskset -c 0-7
PIN="--pin none" run node1 taskset -c 64-71
run auto2
