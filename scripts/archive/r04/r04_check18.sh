#!/bin/bash
# r04: k_random_go back at 1024 threads with the LDS event window, the tag atomics and the ballot prefix counts;
# its parity tests, then C2 Random on Go's stream and C4 against the previous library (abtmp/prev), interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_random_go.py tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
P=KSIM_LIB_PATH=$PWD/abtmp/prev/libksim_hip.so
for i in 1 2 3; do
  one rgo_prev_$i "--policy Random --random-stream go --steps 5 --warmup 1" $P
  one rgo_new_$i "--policy Random --random-stream go --steps 5 --warmup 1"
  one c4_prev_$i "--config c4 --steps 3 --warmup 1" $P
  one c4_new_$i "--config c4 --steps 3 --warmup 1"
done
