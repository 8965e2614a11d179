#!/bin/bash
# r04: L2 (second maxima) back for the wide k_hmemo only -- its parity tests (wide form, C5, shards, stress),
# then C5 with and without it (interleaved) and C5's phase profile.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c5b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_c5.py tests/test_gpu_memo.py tests/test_gpu_hdelay.py tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  one c5_l2_$i "--config c5 --steps 2 --warmup 1"
  one c5_nol2_$i "--config c5 --steps 2 --warmup 1" KSIM_HL2=0
done
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1; grep -o "us/step.*" $O/prof_c5.log
