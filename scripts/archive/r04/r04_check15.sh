#!/bin/bash
# r04: the concurrent groups' reports over one / three / six side streams (tests/test_gpu_report.py).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c15; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; exit $rc
