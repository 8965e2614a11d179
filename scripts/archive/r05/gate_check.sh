#!/bin/bash
# r05: the FGD residency gate -- sweep + mix parity, then C4 A/B (gate default vs KSIM_C4_GATE=0), then the
# default bench order (CPU baseline first) with the gate
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_scan1_mix.py tests/test_gpu_sweep.py > gpurun_out/r05c3/tests.log 2>&1 || { tail -30 gpurun_out/r05c3/tests.log; exit 1; }
tail -2 gpurun_out/r05c3/tests.log
bash scripts/r05/c4_ab.sh r05c3 3 "gate:KSIM_C4_GATE=1" "nogate:KSIM_C4_GATE=0" && \
bash scripts/r05/c4_ab.sh r05c3 2 "cpugate:KSIM_C4_GATE=1"
