#!/bin/bash
# rocprofv3 kernel-trace stats + PMC traffic passes of the bench, into gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit $?
echo "rocprof ok"; find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs cat
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err || exit $?
  echo "pmc $c ok"
done
python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE --out gpurun_out/pmc_traffic.json \
  --workload "${PMC_WORKLOAD:-blocks=10,entries=1000000}" --source "${PMC_SOURCE:-tools/gpu_prof.sh}" | tee gpurun_out/pmc_summary.txt
