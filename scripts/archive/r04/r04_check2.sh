#!/bin/bash
# r04 on one box: the memo / stress / PWR parity tests, then interleaved A/Bs against the r03 library
# (abtmp/r03 via KSIM_LIB_PATH): C2 (k_memo without the end barrier), PWR 500 FGD 500 (the A round
# published early), C4 and C2 run_mode 5 (k_hmemo with L2, KSIM_HL2=0 without), C4's FGD traces one by one.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c2; mkdir -p $O
export TMPDIR=/tmp
R03=KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_hdelay.py tests/test_gpu_pwr.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args-string env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one c2_r03_$i "--steps 10 --warmup 2" $R03
  one c2_r04_$i "--steps 10 --warmup 2"
  one c2_notop_$i "--steps 10 --warmup 2" KSIM_MEMO_TOP=0
done
for i in 1 2; do
  one pf_r03_$i "--steps 5 --warmup 1 --policy PWR_500_FGD_500" $R03
  one pf_r04_$i "--steps 5 --warmup 1 --policy PWR_500_FGD_500"
  one c4_r03_$i "--config c4 --steps 3 --warmup 1" $R03
  one c4_r04_$i "--config c4 --steps 3 --warmup 1"
  one c4_nol2_$i "--config c4 --steps 3 --warmup 1" KSIM_HL2=0
  one rm5_r04_$i "--steps 5 --warmup 1 --run-mode 5"
  one rm5_nol2_$i "--steps 5 --warmup 1 --run-mode 5" KSIM_HL2=0
done
KSIM_PROFILE=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_memo.log 2>&1; grep "memo profile" $O/prof_memo.log
KSIM_PROFILE=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --run-mode 5 > $O/prof_rm5.log 2>&1; grep "hmemo profile" $O/prof_rm5.log
timeout -k 10 300 python -u scripts/c4_fgd_traces.py > $O/c4_traces.log 2>&1; tail -17 $O/c4_traces.log
# ONE cooperative-launch counter pass of the torch-free world-1 bench (round-3 verdict item 2), maps saved
KSIM_MAPS_OUT=$O/maps.txt timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_coop.log 2>&1
echo "pmc coop rc=$?"
grep -A22 Aborted $O/pmc_coop.log | head -24
