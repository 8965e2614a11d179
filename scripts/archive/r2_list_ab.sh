#!/bin/bash
# k_hmemo lane-parallel F list + k_scan1 (with the cluster report): parity with the candidate library,
# phase profile, interleaved timing, C4 policy groups with and without k_scan1.
# Usage: bash scripts/r2_list_ab.sh base.so cand.so
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lab; mkdir -p $O
V=${@: -1}
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $V $LIB
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread ${PARITY_TESTS:-tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_memo.py tests/test_gpu_report.py tests/test_gpu_dotprod.py tests/test_gpu_sweep.py tests/test_gpu_c5.py} -k "not (c5 and (full or sharded))" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
bash scripts/ab_configs.sh "--run-mode 5 --steps 3;--config c5 --steps 1 --warmup 0;--config c4 --steps 2" "$@" || exit 1
cp $V $LIB
timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4_groups.log 2>&1; tail -1 $O/c4_groups.log
KSIM_SCAN1=0 timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4_groups_noscan1.log 2>&1; tail -1 $O/c4_groups_noscan1.log
