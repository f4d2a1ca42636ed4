#!/bin/bash
# Config 5 alone under rocprofv3: kernel trace (+ stats), then FETCH_SIZE and WRITE_SIZE passes,
# each its own run; summaries of the rocpd databases by tools/rpd_summary.py.
set -e
mkdir -p gpurun_out/lkprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=/tmp/c5w
C="python3 tools/c45_prof.py --workdir $W --cfg4 0 --cfg5 1 --cfg5-steps 10"
timeout -k 10 300 $C > gpurun_out/lkprof/gen.json 2> gpurun_out/lkprof/gen.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof/kt -o lk -- $C > gpurun_out/lkprof/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/lkprof/fetch -o lk -- $C > gpurun_out/lkprof/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/lkprof/write -o lk -- $C > gpurun_out/lkprof/write.log 2>&1
for d in kt fetch write; do
  db=$(find gpurun_out/lkprof/$d -name "*.db" | head -1)
  echo "== $d $db"
  if [ $d = kt ]; then python3 tools/rpd_summary.py stats "$db" > gpurun_out/lkprof/${d}_stats.txt; cat gpurun_out/lkprof/${d}_stats.txt; fi
  python3 tools/rpd_summary.py pmc "$db" lookup_ > gpurun_out/lkprof/${d}_lookup.txt || true
done
