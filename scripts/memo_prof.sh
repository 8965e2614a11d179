#!/bin/bash
# k_memo phase profile (KSIM_PROFILE=1) and owner/hand-off trace (KSIM_PROFILE=2) of the C2 bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
KSIM_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/memo_prof.log 2>&1 || exit $?
grep "memo profile" gpurun_out/memo_prof.log
KSIM_PROFILE=2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/memo_trace.log 2>&1 || exit $?
grep "memo trace" gpurun_out/memo_trace.log
