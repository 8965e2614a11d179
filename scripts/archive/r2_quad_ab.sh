#!/bin/bash
# frag_F_quad changes (k_hmemo, k_replay FGD / PWR+FGD): parity with the variant, then interleaved timing.
# Usage: bash scripts/r2_quad_ab.sh base.so variant.so
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qab; mkdir -p $O
V=${@: -1}
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $V $LIB
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_memo.py tests/test_gpu_fuzz.py tests/test_gpu_pwr.py tests/test_gpu_parity.py tests/test_gpu_c5.py tests/test_gpu_sweep.py -k "not (c5 and (full or million or 1m))" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
cp $V $LIB
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
bash scripts/ab_configs.sh "--run-mode 5 --steps 3;--config c5 --steps 1 --warmup 0;--run-mode 2 --steps 3;--policy PWR_500_FGD_500 --steps 3;--config c4 --steps 2" "$@" || exit 1
cp $V $LIB
