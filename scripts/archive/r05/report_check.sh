#!/bin/bash
# r05: the one-pass report scan -- report / log-contract / sweep parity, then the C4 timeline + kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c5
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_report.py tests/test_gpu_log_contract.py tests/test_gpu_scan1_mix.py tests/test_gpu_sweep.py \
  > gpurun_out/r05c5/tests.log 2>&1 || { tail -30 gpurun_out/r05c5/tests.log; exit 1; }
tail -2 gpurun_out/r05c5/tests.log
bash scripts/r05/c4_prof.sh r05c5
