#!/bin/bash
# r04 A/B on one box, interleaved: the r03 library (abtmp/r03, KSIM_LIB_PATH) against this tree's, with
# k_memo's early owner path on and off (KSIM_MEMO_EARLY); the early path's trace (KSIM_PROFILE=2); then ONE
# cooperative FETCH_SIZE counter pass of the torch-free world-1 bench, with the process's maps saved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04ab2; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/b_$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']), d.get('hip_runtime', {}).get('hip'))"
}
for i in 1 2 3; do
  one r03_$i KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
  one early1_$i KSIM_MEMO_EARLY=1
  one early0_$i KSIM_MEMO_EARLY=0
done
KSIM_PROFILE=2 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
grep "memo trace\|memo early" $O/trace.log
KSIM_MAPS_OUT=$O/maps.txt timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_coop.log 2>&1
echo "pmc coop rc=$?"
grep -A22 Aborted $O/pmc_coop.log | head -24
