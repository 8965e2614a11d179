#!/bin/bash
# r05: new k_hmemo variant tests + mix, C5 A/B against the r04 library (same box), the C4 rank shares at one
# workgroup per replica
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c10; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py::test_hmemo_list_and_table_forms tests/test_gpu_scan1_mix.py tests/test_gpu_report.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in r05 r04; do
    if [ $v = r04 ]; then export KSIM_LIB_PATH=$PWD/abtmp_r04/libksim_hip.so; else unset KSIM_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${v}_$i.json')); print('c5 $v $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
unset KSIM_LIB_PATH
sed -i 's#r05c6#r05c10#' scripts/r05/c4_shares.sh
bash scripts/r05/c4_shares.sh
# C4: the 6-wave k_scan1_mix (this tree) against the 5-wave library of the previous commit (abtmp_r05a)
bash scripts/r05/c4_ab.sh r05c10 2 "w6:KSIM_SCAN1_MIX=1" "w5:KSIM_LIB_PATH=$PWD/abtmp_r05a/libksim_hip.so"
