#!/bin/bash
# Grid-plan / path sweep of the config-2 search on one GPU: one block set generated
# once, then bench.py under each setting (kernel p50 from the deferred HIP events).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
W=/tmp/tsg_sweep
SETTINGS="${1:-base PER_CU=2 PER_CU=3 PER_CU=6 PER_CU=8 PER_CU=12}"
for st in $SETTINGS; do
  envs=()
  [ "$st" != base ] && for kv in ${st//,/ }; do envs+=("TSG_$kv"); done
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --cpu-baseline 0 --limit-steps 0 \
    --workdir $W ${BENCH_ARGS:-} > gpurun_out/sweep_$st.json 2> gpurun_out/sweep_$st.err
  rc=$?
  [ $rc -eq 0 ] || { echo "$st rc=$rc"; tail -5 gpurun_out/sweep_$st.err; exit $rc; }
  python3 - "$st" gpurun_out/sweep_$st.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d["latency_us"]["kernel"]; s = d["latency_us"]["step"]
print(f"{sys.argv[1]:>14}: kernel p10/p50/p90 {k['p10']:.1f}/{k['p50']:.1f}/{k['p90']:.1f} us  step p50 {s['p50']:.1f} us  "
      f"frac {d['roofline']['frac']:.3f}  value {d['value']/1e9:.1f} G/s  matches {d['config']['matches_per_gpu']}", flush=True)
PY
done
