#!/bin/bash
# k_pmemo phase profile (KSIM_PROFILE=1) and exchange trace (KSIM_PROFILE=2) of the C2 bench on run_mode 6.
mkdir -p gpurun_out
export TMPDIR=/tmp
KSIM_PROFILE=1 timeout -k 10 300 python bench.py --run-mode 6 --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pm_prof.log 2>&1 || exit $?
grep "pmemo profile" gpurun_out/pm_prof.log
KSIM_PROFILE=2 timeout -k 10 300 python bench.py --run-mode 6 --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pm_trace.log 2>&1 || exit $?
grep "pmemo trace" gpurun_out/pm_trace.log
