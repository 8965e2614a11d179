#!/bin/bash
# r04: the launch gate for the concurrent groups (the short groups wait until every k_hmemo workgroup is
# resident).  Parity (sweep, report), then C4 as bench.py runs it by default (CPU baseline first) with and
# without the gate (KSIM_GATE=0), interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c20; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one c4_gate_$i "--config c4"
  one c4_nogate_$i "--config c4" KSIM_GATE=0
done
