#!/bin/bash
# r05: PWR + FGD with the A round out before the FGD evaluation -- PWR parity (incl. the memo's version wrap, the
# fuzz's PWR cases, the report), then C2 PWR 500 FGD 500 / PWR against the previous library (abtmp_prev)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c17; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pwr.py tests/test_gpu_fuzz.py tests/test_gpu_report.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in new prev; do
    unset KSIM_LIB_PATH
    [ $v = prev ] && export KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so
    timeout -k 10 200 python -u bench.py --policy "PWR 500 FGD 500" --no-cpu-baseline --steps 5 --warmup 1 > $OUT/pf_${v}_$i.json 2> $OUT/pf_${v}_$i.err || { tail -5 $OUT/pf_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/pf_${v}_$i.json')); print('pwr500fgd500 $v $i', round(d['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
