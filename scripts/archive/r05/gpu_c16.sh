#!/bin/bash
# r05: pruning only in the large-table k_hmemo instantiation -- memo tests, C2 run_mode 5 and C4 against the
# previous library (abtmp_prev), one box
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c16; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_sweep.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in new prev; do
    unset KSIM_LIB_PATH
    [ $v = prev ] && export KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so
    timeout -k 10 200 python -u bench.py --run-mode 5 --no-cpu-baseline --steps 5 --warmup 1 > $OUT/rm5_${v}_$i.json 2> $OUT/rm5_${v}_$i.err || { tail -5 $OUT/rm5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/rm5_${v}_$i.json')); print('rm5 $v $i', round(d['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
unset KSIM_LIB_PATH
bash scripts/r05/c4_ab.sh r05c16 2 "new:KSIM_SCAN1_MIX=1" "prev:KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so"
