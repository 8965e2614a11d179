#!/bin/bash
# VALU issue fraction of the bench's dominant kernel (FGD is VALU-bound, report it
# beside the HBM fraction). One --pmc pass of its own (SQ_INSTS_VALU, SQ_WAVES, GRBM_GUI_ACTIVE).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_valu
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -20 $OUT/pmc.log; exit 1; }
find $OUT/pmc -name "*counter_collection.csv" -exec cp {} $OUT/counter_collection.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/kt.log 2>&1 || { echo "kt pass failed rc=$?"; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -c 600 $OUT/counter_collection.csv
