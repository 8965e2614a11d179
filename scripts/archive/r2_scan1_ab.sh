#!/bin/bash
# k_hmemo octet F + k_scan1: parity with the candidate library, then interleaved timing.
# Usage: bash scripts/r2_scan1_ab.sh base.so oct.so cur.so   (cur = the candidate, last)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sab; mkdir -p $O
V=${@: -1}
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $V $LIB
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread ${PARITY_TESTS:-tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_memo.py tests/test_gpu_dotprod.py tests/test_gpu_sweep.py tests/test_gpu_c5.py} -k "not (c5 and (full or sharded))" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
for pol in BestFit GpuClustering; do for s1 in 0 1; do
  KSIM_SCAN1=$s1 timeout -k 10 200 python3 bench.py --policy $pol --wgs 1 --steps 3 --no-cpu-baseline > $O/b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$pol K=1 KSIM_SCAN1=$s1 dev ms %.2f'%d['device_ms_per_step'])"
done; done
bash scripts/ab_configs.sh "--config c4 --steps 2;--run-mode 5 --steps 3;--config c5 --steps 1 --warmup 0" "$@" || exit 1
cp $V $LIB
timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4_groups.log 2>&1; tail -1 $O/c4_groups.log
KSIM_SCAN1=0 timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4_groups_noscan1.log 2>&1; tail -1 $O/c4_groups_noscan1.log
