#!/bin/bash
# r05: k_hmemo's F items round robin over the F waves -- memo / hdelay / sweep / C5 parity, then C5, C2 run_mode 5
# and C4 against the previous library (abtmp_prev), one box
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c18; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_hdelay.py tests/test_gpu_sweep.py tests/test_gpu_c5.py tests/test_gpu_scan1_mix.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in new prev; do
    unset KSIM_LIB_PATH
    [ $v = prev ] && export KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    timeout -k 10 200 python -u bench.py --run-mode 5 --no-cpu-baseline --steps 5 --warmup 1 > $OUT/rm5_${v}_$i.json 2> $OUT/rm5_${v}_$i.err || { tail -5 $OUT/rm5_${v}_$i.err; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/c5_${v}_$i.json')); b=json.load(open('$OUT/rm5_${v}_$i.json')); print('$v $i c5', round(a['ms_per_step'],1), 'rm5', round(b['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
unset KSIM_LIB_PATH
bash scripts/r05/c4_ab.sh r05c18 2 "new:KSIM_SCAN1_MIX=1" "prev:KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so"
