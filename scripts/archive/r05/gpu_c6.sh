#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c6
KSIM_PROFILE=1 timeout -k 10 300 python -u scripts/r05/hmemo_phases.py default gpuspec10 gpuspec33 > gpurun_out/r05c6/phases.log 2>&1 || { tail -5 gpurun_out/r05c6/phases.log; exit 1; }
grep -E "trace|hmemo profile" gpurun_out/r05c6/phases.log
bash scripts/r05/c4_shares.sh
