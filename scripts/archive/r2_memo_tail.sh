#!/bin/bash
# k_memo wave_F fold without the zero-padding batches: parity (k_memo paths), then C2 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tail; mkdir -p $O
cp abtmp/tail.so kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_memo.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "memo or full_openb_fgd or FGD" > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
for r in 1 2 3; do bash scripts/ab_configs.sh "--steps 10" abtmp/head.so abtmp/tail.so | grep dev || exit 1; done
