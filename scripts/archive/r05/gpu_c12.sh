#!/bin/bash
# r05: the spec divisions as corrected products -- parity of the cheap policies, C4 and C2 BestFit / DotProd
# A/B against the previous library (abtmp_r05b)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c12; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_dotprod.py tests/test_gpu_scan1_mix.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/r05/c4_ab.sh r05c12 2 "new:KSIM_SCAN1_MIX=1" "old:KSIM_LIB_PATH=$PWD/abtmp_r05b/libksim_hip.so" || exit 1
for pol in BestFit DotProd; do
  for v in new old; do
    if [ $v = old ]; then export KSIM_LIB_PATH=$PWD/abtmp_r05b/libksim_hip.so; else unset KSIM_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --policy $pol --no-cpu-baseline --steps 5 --warmup 1 > $OUT/c2_${pol}_$v.json 2> $OUT/c2_${pol}_$v.err || { tail -5 $OUT/c2_${pol}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_${pol}_$v.json')); print('c2 $pol $v', round(d['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
