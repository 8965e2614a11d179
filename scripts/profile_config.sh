#!/bin/bash
# Counter-backed roofline of one bench configuration (run on a gpurun box):
#   1. rocprofv3 --kernel-trace --stats   -> every kernel's dispatches and durations
#   2. --pmc FETCH_SIZE                   -> HBM read bytes per dispatch (x2, gfx950 correction)
#   3. --pmc WRITE_SIZE                   -> HBM write bytes per dispatch
#   4. --pmc SQ_INSTS_VALU + the fp64 ADD / MUL / FMA counts + SQ_WAVES + GRBM_GUI_ACTIVE
# (separate passes: MI355X_MICROARCH.md rocprofv3 section; never --pmc with sys/runtime traces)
# then scripts/pmc_summary.py -> <out>/pmc.json.  Usage: bash scripts/profile_config.sh NAME [bench args...]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
# plain launches of the same grids (rocprofv3 7.2 faults in the HIP runtime's exit handlers after a cooperative
# launch, one runtime in the process or two: DESIGN.md §3; the grid size
# is still bounded by the occupancy cap, and the kernels are the same)
export KSIM_COOP=0
NAME=$1; shift
OUT=gpurun_out/prof/$NAME
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline $*"
echo "== $NAME: $BENCH ($(date +%T))"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $BENCH \
  > $OUT/kt.log 2>&1 || { echo "kernel-trace pass failed rc=$?"; tail -20 $OUT/kt.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $BENCH \
  > $OUT/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed rc=$?"; tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $BENCH \
  > $OUT/write.log 2>&1 || { echo "WRITE_SIZE pass failed rc=$?"; tail -20 $OUT/write.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
  SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- python3 $BENCH \
  > $OUT/valu.log 2>&1 || { echo "VALU pass failed rc=$?"; tail -20 $OUT/valu.log; exit 1; }
python3 scripts/pmc_summary.py $OUT "$*" > $OUT/pmc.json || exit 1
# keep the summaries small: the per-kernel stats and the json travel back, the raw traces stay here
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/kt $OUT/fetch $OUT/write $OUT/valu
python3 -c "
import json; d = json.load(open('$OUT/pmc.json'))
k = d['dominant']; print('$NAME', k['kernel'], 'ms %.3f' % (k['mean_duration_ns'] / 1e6), 'HBM MB/dispatch %.1f' % (k.get('hbm_bytes_per_dispatch', 0) / 1e6),
      'VALU frac %.3f' % k.get('valu_frac', 0), 'fp64 share %.3f' % k.get('f64_share', 0))"
