#!/bin/bash
# r05: C5 with 8 F waves in the wide k_hmemo (this tree) against 7 (abtmp_prev), one box, interleaved; the wide
# form's parity first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c15; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py -k "wide" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in fw8 fw7; do
    unset KSIM_LIB_PATH
    [ $v = fw7 ] && export KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$i.json')); print('c5 $v $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
