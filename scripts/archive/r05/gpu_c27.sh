#!/bin/bash
# r05: the wide k_hmemo without the L2 code -- k_hmemo parity (memo forms, C5 prefix + properties, hand-over stress),
# then C5 against the library before (abtmp_bis/cur) and r03's, interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c27; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_c5.py tests/test_gpu_hdelay.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do
  for v in new cur r03; do
    unset KSIM_LIB_PATH
    case $v in r03) export KSIM_LIB_PATH=$PWD/abtmp_r03/libksim_hip.so;; cur) export KSIM_LIB_PATH=$PWD/abtmp_bis/cur/libksim_hip.so;; esac
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { echo "c5 $v $i failed"; tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$i.json')); print('c5 $v $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
