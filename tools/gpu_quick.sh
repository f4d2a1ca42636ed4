set -u
mkdir -p gpurun_out
TSG_STAMPS=1 TSG_TRACE=1 timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/stamps.json 2> gpurun_out/stamps.err || exit $?
grep "stamps" gpurun_out/stamps.err | tail -4
TSG_TRACE=1 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/trace.json 2> gpurun_out/trace.err || exit $?
grep "\[tsg\]" gpurun_out/trace.err | tail -4
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
