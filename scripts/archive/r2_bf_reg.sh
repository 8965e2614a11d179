#!/bin/bash
# Branch-free class-pass filter in k_hmemo (bf) and k_scan1 with VGPR-resident records (KSIM_SCAN1=2):
# parity with bf.so, then A/B timing.  Usage: bash scripts/r2_bf_reg.sh base.so bf.so
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/bfr; mkdir -p $O
V=${@: -1}
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $V $LIB
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_memo.py tests/test_gpu_fuzz.py tests/test_gpu_c5.py tests/test_gpu_parity.py tests/test_gpu_sweep.py -k "hmemo or FGD or prefix or step_kernel or single_workgroup or full_paper" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
bash scripts/ab_configs.sh "--run-mode 5 --steps 3;--config c5 --steps 1 --warmup 0" "$@" || exit 1
cp $V $LIB
for r in 1 2; do for m in 1 2; do
  KSIM_SCAN1=$m timeout -k 10 300 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > $O/b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('c4 KSIM_SCAN1=$m dev ms %.2f'%d['device_ms_per_step'], flush=True)"
done; done
for m in 2 1; do KSIM_SCAN1=$m timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4g_$m.log 2>&1; echo "KSIM_SCAN1=$m $(tail -1 $O/c4g_$m.log)"; done
