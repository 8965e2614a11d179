#!/bin/bash
# r04: k_memo with one granule poller per workgroup (LDS hand-over to the other waves) against the r03
# library, the k_hmemo refresh-list prefetch (KSIM_HPF) on C4 / run_mode 5, the profiler exit fault with the
# device released before exit (KSIM_DEVICE_RESET=1).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c3; mkdir -p $O
export TMPDIR=/tmp
R03=KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_hdelay.py -k "memo or c2_delays" > $O/tests.log 2>&1
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
done
for i in 1 2; do
  one c4_hpf0_$i "--config c4 --steps 3 --warmup 1"
  one c4_hpf1_$i "--config c4 --steps 3 --warmup 1" KSIM_HPF=1
  one c4_hpf3_$i "--config c4 --steps 3 --warmup 1" KSIM_HPF=3
  one rm5_hpf0_$i "--steps 5 --warmup 1 --run-mode 5"
  one rm5_hpf1_$i "--steps 5 --warmup 1 --run-mode 5" KSIM_HPF=1
done
KSIM_PROFILE=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_memo.log 2>&1; grep "memo profile" $O/prof_memo.log
KSIM_DEVICE_RESET=1 KSIM_MAPS_OUT=$O/maps.txt timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_coop.log 2>&1
echo "pmc coop (device reset before exit) rc=$?"
grep -A22 Aborted $O/pmc_coop.log | head -24
ls $O/fetch | head
