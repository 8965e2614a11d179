#!/bin/bash
# Round profile of the bench workload (run on a gpurun box):
#   1. rocprofv3 --kernel-trace --stats     -> the dominant kernel's duration (k_memo; must agree with bench.py's hipEvents)
#   2. rocprofv3 --pmc FETCH_SIZE           -> HBM read bytes per dispatch (x2, gfx950 correction)
#   3. rocprofv3 --pmc WRITE_SIZE           -> HBM write bytes per dispatch
# (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; no --pmc with sys/runtime traces)
#   4. the default bench line (with cpu_baseline)
# Writes gpurun_out/prof_round/{kt,fetch,write}/..., gpurun_out/prof_round/pmc.json, gpurun_out/prof_round/bench.json
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_round
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $BENCH \
  > $OUT/kt.log 2>&1 || { echo "kernel-trace pass failed rc=$?"; tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $BENCH \
  > $OUT/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed rc=$?"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $BENCH \
  > $OUT/write.log 2>&1 || { echo "WRITE_SIZE pass failed rc=$?"; tail -20 $OUT/write.log; exit 1; }
python3 scripts/pmc_summary.py $OUT > $OUT/pmc.json || exit 1
cat $OUT/pmc.json
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
