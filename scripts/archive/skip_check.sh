#!/bin/bash
# the dead-class skip: memoised-path parity, then the C2 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_pmemo.py tests/test_gpu_fuzz.py "$@" > gpurun_out/skip_tests.log 2>&1
rc=$?
tail -3 gpurun_out/skip_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/skip_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/skip_bench.log 2>&1
rc=$?
tail -1 gpurun_out/skip_bench.log | cut -c1-420
exit $rc
