#!/bin/bash
# GPU test suite on a gpurun box: one pytest process, per-test timeout, log under gpurun_out/.
# Usage: bash scripts/gpu_tests.sh [pytest selection args...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest -v --durations=40 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu "$@" \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
exit $rc
