#!/bin/bash
# k_pmemo on a gpurun box: its parity tests, then the C2 bench on run_mode 6, its phase profile and trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_pmemo.py "$@" > gpurun_out/pm_tests.log 2>&1
rc=$?
tail -4 gpurun_out/pm_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pm_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --run-mode 6 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pm_bench.log 2>&1
rc=$?
tail -1 gpurun_out/pm_bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
bash scripts/archive/pm_prof.sh
