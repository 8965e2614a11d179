#!/bin/bash
# HBM traffic and VALU instructions of k_replay for one non-FGD policy at C2 (separate --pmc passes).
# Usage: bash scripts/profile_policy.sh BestFit
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
POL=${1:-BestFit}
OUT=gpurun_out/prof_$POL
mkdir -p $OUT
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --policy $POL"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $B > $OUT/kt.log 2>&1 || { echo "kt rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B > $OUT/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- python3 $B > $OUT/valu.log 2>&1 || { echo "valu rc=$?"; exit 1; }
echo done
