#!/bin/bash
# r04 k_memo without the end-of-step barrier: its parity tests and the delay stress, then the C2 bench
# interleaved with the r03 library (abtmp/r03, KSIM_LIB_PATH) on the same box.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04memo; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_hdelay.py tests/test_gpu_pwr.py -k "memo or c2_delays or pwr or PWR" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/b_$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one r03_$i KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
  one r04_$i
done
onep() {  # PWR 500 FGD 500
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --policy "PWR 500 FGD 500" > $O/p_$tag.json 2> $O/p_$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench pwr $tag rc=$rc"; tail -5 $O/p_$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/p_$tag.json').read().strip().splitlines()[-1]); print('PWR+FGD $tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  onep r03_$i KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
  onep r04_$i
done
KSIM_PROFILE=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/prof.log 2>&1; grep "memo profile" $O/prof.log
timeout -k 10 200 python -u scripts/c4_fgd_traces.py > $O/c4_traces.log 2>&1; cat $O/c4_traces.log | tail -17
