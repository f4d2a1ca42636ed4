#!/bin/bash
# Config-5 count-pass A/B (TSG_LK_OCC = 6 / 7 / 8 waves, 17 = 7 waves + non-temporal ids and
# counts; TSG_LK_PAIR) on one box (LK_VARIANTS="occ_pair[_slotmajor[_hostsize[_tr]]] ...", LK_TESTS="occ ..."):
# cfg5 device time per variant, then the lookup parity tests under the fastest variants.
set -e
mkdir -p gpurun_out
W=/tmp/c5w
for v in ${LK_VARIANTS:-6_0 7_0 8_0 7_1 6_0}; do
  set -- ${v//_/ }
  TSG_LK_TR=${5:-2} TSG_LK_HOSTSIZE=${4:-0} TSG_LK_SLOTMAJOR=${3:-1} TSG_LK_OCC=$1 TSG_LK_PAIR=$2 timeout -k 10 400 python3 -u tools/c45_prof.py --workdir $W --cfg4 0 --cfg5 1 --cfg5-steps 20 \
    > gpurun_out/lk_o$1_p$2_s${3:-1}_h${4:-0}_t${5:-2}.json 2> gpurun_out/lk_o$1_p$2_s${3:-1}_h${4:-0}_t${5:-2}.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/lk_o$1_p$2_s${3:-1}_h${4:-0}_t${5:-2}.json').read().strip().splitlines()[-1])['cfg5']; print('occ $1 pair $2 slotmajor ${3:-1} hostsize ${4:-0} tr ${5:-2}', round(d['device_ms'],3), 'ms hits', d['hits_rank0'])"
done
for o in ${LK_TESTS:-7 8}; do
  TSG_LK_OCC=$o timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lookup.py > gpurun_out/lk_test_o$o.txt 2>&1
  tail -1 gpurun_out/lk_test_o$o.txt
done
