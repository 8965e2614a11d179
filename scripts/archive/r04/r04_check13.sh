#!/bin/bash
# r04: k_hmemo keys in a node-grouped layout ([Npad/4][Cmax][4]: a refresh's key stores cover 8 cache lines
# per wave instead of 64).  Parity of every k_hmemo path, then A/B against the previous library (abtmp/prev),
# interleaved: run_mode 5, C5, C4.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_hdelay.py tests/test_gpu_memo.py tests/test_gpu_c5.py tests/test_gpu_shard.py tests/test_gpu_sweep.py \
  tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
P=KSIM_LIB_PATH=$PWD/abtmp/prev/libksim_hip.so
for i in 1 2; do
  one rm5_prev_$i "--run-mode 5 --steps 10 --warmup 2" $P
  one rm5_new_$i "--run-mode 5 --steps 10 --warmup 2"
  one c5_prev_$i "--config c5 --steps 2 --warmup 1" $P
  one c5_new_$i "--config c5 --steps 2 --warmup 1"
  one c4_prev_$i "--config c4 --steps 3 --warmup 1" $P
  one c4_new_$i "--config c4 --steps 3 --warmup 1"
done
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1; grep -o "us/step.*" $O/prof_c5.log
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_rm5.log 2>&1; grep -o "us/step.*" $O/prof_rm5.log
