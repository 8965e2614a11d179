#!/bin/bash
# r04: C4's slow runs serialise the side streams (KSIM_GROUP_TIMES: every stream ends with the FGD one).  Side
# streams with an all-CU mask (KSIM_SIDE_CUMASK=1: a hardware queue each) against the default, C4 as bench.py
# runs it by default, interleaved; then the concurrent-path parity tests with the mask.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c22; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 1 0; do
    KSIM_SIDE_CUMASK=$v KSIM_GROUP_TIMES=1 timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/c4_m${v}_$i.json 2> $O/c4_m${v}_$i.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $O/c4_m${v}_$i.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('$O/c4_m${v}_$i.json').read().strip().splitlines()[-1]); print('c4 cumask=$v run $i: %.3f ms' % d['ms_per_step'])"
    grep "group times" $O/c4_m${v}_$i.err | tail -1
  done
done
KSIM_SIDE_CUMASK=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; exit $rc
