mkdir -p gpurun_out
W=/tmp/shimwd; mkdir -p $W
TSG_PROF=1 timeout -k 10 300 python tools/shim_probe.py --limit 20 --workdir $W > gpurun_out/shim20.out 2> gpurun_out/shim20.err && \
TSG_PROF=1 timeout -k 10 300 python tools/shim_probe.py --limit 0 --workdir $W > gpurun_out/shim0.out 2> gpurun_out/shim0.err
rc=$?; cat gpurun_out/shim20.out gpurun_out/shim0.out; grep "prof" gpurun_out/shim20.err gpurun_out/shim0.err; exit $rc
