#!/bin/bash
# r04: k_hmemo's group keys scored by the F waves (LDS atomics) -- the k_hmemo parity and stress tests, then
# the r03 library (abtmp/r03, KSIM_LIB_PATH) against this tree's, interleaved: run_mode 5 at C2, C4, C5.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_hdelay.py tests/test_gpu_memo.py tests/test_gpu_c5.py tests/test_gpu_shard.py tests/test_gpu_sweep.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
R03=KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
for i in 1 2; do
  one rm5_r03_$i "--run-mode 5 --steps 10 --warmup 2" $R03
  one rm5_new_$i "--run-mode 5 --steps 10 --warmup 2"
  one c4_r03_$i "--config c4 --steps 10 --warmup 2" $R03
  one c4_new_$i "--config c4 --steps 10 --warmup 2"
done
one c5_r03 "--config c5 --steps 2 --warmup 1" $R03
one c5_new "--config c5 --steps 2 --warmup 1"
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1; grep -o "us/step.*" $O/prof_c5.log
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_rm5.log 2>&1; grep -o "us/step.*" $O/prof_rm5.log
# PWR + FGD (k_replay<7>): the phase profile, then workgroups per replica
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --policy "PWR 500 FGD 500" --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_pf.log 2>&1; grep -o "ksim profile.*" $O/prof_pf.log
for k in 25 16 10 32; do one pf_k$k "--policy PWR_500_FGD_500 --wgs $k --steps 5 --warmup 1"; done
# C4: the concurrent groups on no more side streams than hardware queues (default) vs six (r03's mapping shape)
for i in 1 2; do
  one c4_q4_$i "--config c4 --steps 3 --warmup 1"
  one c4_q6_$i "--config c4 --steps 3 --warmup 1" KSIM_SIDE_STREAMS=6
done
