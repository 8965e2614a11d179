#!/bin/bash
# k_hmemo variant check: parity with the variant library in place, phase profiles and interleaved
# timing against the baseline.  Usage: bash scripts/r2_hmemo_ab.sh base.so variant.so [more.so]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hab; mkdir -p $O
V=${@: -1}
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $V $LIB
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_memo.py tests/test_gpu_fuzz.py tests/test_gpu_c5.py tests/test_gpu_sweep.py -k "hmemo or FGD or prefix or step_kernel or sweep" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
for so in "$@"; do cp $so $LIB
  KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
done
bash scripts/ab_configs.sh "--run-mode 5 --steps 3;--config c4 --steps 2;--config c5 --steps 1 --warmup 0" "$@" || exit 1
cp $V $LIB
