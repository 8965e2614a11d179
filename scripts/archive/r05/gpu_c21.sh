#!/bin/bash
# r05: PWR + FGD in one round per step (guessed NormalizeScore ranges, miss round, owner re-evaluation) -- PWR parity
# (K auto / 1 / 4, the memo and its version wrap, deletions, the report, the fuzz), then C2 PWR 500 FGD 500 against the
# previous library (abtmp_pf0), and one KSIM_PROFILE run for the phase split and the miss / re-evaluation rates
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r05c21}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pwr.py tests/test_gpu_fuzz.py tests/test_gpu_report.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  for v in new prev; do
    unset KSIM_LIB_PATH
    [ $v = prev ] && export KSIM_LIB_PATH=$PWD/abtmp_pf0/libksim_hip.so
    timeout -k 10 200 python -u bench.py --policy "PWR 500 FGD 500" --no-cpu-baseline --steps 5 --warmup 1 > $OUT/pf_${v}_$i.json 2> $OUT/pf_${v}_$i.err || { tail -5 $OUT/pf_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/pf_${v}_$i.json')); print('pwr500fgd500 $v $i', round(d['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
unset KSIM_LIB_PATH
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --policy "PWR 500 FGD 500" --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pf_prof.json 2> $OUT/pf_prof.err || { tail -5 $OUT/pf_prof.err; exit 1; }
grep "ksim profile" $OUT/pf_prof.err | tail -1 | tee -a $OUT/summary.txt
