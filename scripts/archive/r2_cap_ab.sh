#!/bin/bash
# k_scan1 built for eight workgroups per CU (64 VGPRs) against the head: parity, then C4 timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cap; mkdir -p $O
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp abtmp/cap.so $LIB
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_dotprod.py -k "single_workgroup or full_paper or K1" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
bash scripts/ab_configs.sh "--config c4 --steps 3" abtmp/head.so abtmp/cap.so || exit 1
for so in head cap; do cp abtmp/$so.so $LIB; timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4g_$so.log 2>&1; echo "$so $(tail -1 $O/c4g_$so.log)"; done
