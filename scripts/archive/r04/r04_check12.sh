#!/bin/bash
# r04 timing experiment (not a product path): how much of a k_hmemo step the bulk's key stores cost.  A library
# built with KSIM_HPF bit 8 skipping the class update's HBM key stores (abtmp/dbg, wrong decisions by
# construction) against the same library without the bit, C5 and run_mode 5, interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c12; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
L=KSIM_LIB_PATH=$PWD/abtmp/dbg/libksim_hip.so
for i in 1 2; do
  one c5_st_$i "--config c5 --steps 2 --warmup 1" $L
  one c5_nost_$i "--config c5 --steps 2 --warmup 1" $L KSIM_HPF=9
  one rm5_st_$i "--run-mode 5 --steps 10 --warmup 2" $L
  one rm5_nost_$i "--run-mode 5 --steps 10 --warmup 2" $L KSIM_HPF=9
done
