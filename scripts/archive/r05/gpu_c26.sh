#!/bin/bash
# r05: where the wide k_hmemo lost its r03 time -- C5 on the r03 library, five r04 commits' libraries (abtmp_bis/<commit>)
# and the current one, interleaved on one box
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c26; mkdir -p $OUT
for i in 1 2; do
  for v in r03 002b9cb 2be3f6b 43eef31 0168863 688b12b cur; do
    unset KSIM_LIB_PATH
    case $v in r03) export KSIM_LIB_PATH=$PWD/abtmp_r03/libksim_hip.so;; cur) ;; *) export KSIM_LIB_PATH=$PWD/abtmp_bis/$v/libksim_hip.so;; esac
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { echo "c5 $v $i failed"; tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$i.json')); print('c5 $v $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
