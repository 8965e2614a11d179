#!/bin/bash
# r05: C5 with the F-list pruning in the wide form (KSIM_HPRUNE=-1) against without (default 64: off at T = 35),
# the previous library (abtmp_r05c) and r03's (abtmp_r03), one box, interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c13; mkdir -p $OUT
for i in 1 2; do
  for v in prune noprune prev r03; do
    unset KSIM_LIB_PATH KSIM_HPRUNE
    case $v in prune) export KSIM_HPRUNE=-1;; prev) export KSIM_LIB_PATH=$PWD/abtmp_r05c/libksim_hip.so;; r03) export KSIM_LIB_PATH=$PWD/abtmp_r03/libksim_hip.so;; esac
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$i.json')); print('c5 $v $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
