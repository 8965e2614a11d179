#!/bin/bash
# r04: which concurrent group stretches in C4's slow runs: KSIM_GROUP_TIMES=1 (fork -> each side stream's end),
# C4 as bench.py runs it by default (CPU baseline first), four runs; then the concurrent-path parity tests.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c21; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  KSIM_GROUP_TIMES=1 timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/c4_$i.json 2> $O/c4_$i.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $O/c4_$i.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/c4_$i.json').read().strip().splitlines()[-1]); print('c4_$i: %.3f ms' % d['ms_per_step'])"
  grep "group times" $O/c4_$i.err | tail -2
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; exit $rc
