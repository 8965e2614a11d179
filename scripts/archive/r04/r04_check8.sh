#!/bin/bash
# r04: k_hmemo with more F waves (fewer class waves) for replicas with more than 64 typical pods (KSIM_HFW):
# the sweep's parity at 9, then C4 at 7 (r03's split) / 8 / 9 / 10, interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c8; mkdir -p $O
export TMPDIR=/tmp
KSIM_HFW=9 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_hdelay.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  for f in 7 8 9 10; do one c4_fw${f}_$i "--config c4 --steps 3 --warmup 1" KSIM_HFW=$f; done
done
