#!/bin/bash
# r05: the merged cheap-policy launch (k_scan1_mix) -- targeted GPU tests, then C4 interleaved A/B:
# mix (default) against KSIM_SCAN1_MIX=0 (one k_scan1 launch per policy, r04), with side-stream ends.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_scan1_mix.py tests/test_gpu_parity.py -k "mix or launch or tags or single_workgroup or reserve" \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2 3; do
  for v in mix old; do
    if [ $v = old ]; then export KSIM_SCAN1_MIX=0; else unset KSIM_SCAN1_MIX; fi
    KSIM_GROUP_TIMES=1 timeout -k 10 240 python -u bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1 \
      > $OUT/c4_${v}_$i.json 2> $OUT/c4_${v}_$i.err || { echo "bench $v $i failed"; tail -5 $OUT/c4_${v}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/c4_${v}_$i.json')); print('$v', $i, round(d['ms_per_step'],2), round(d['device_ms_per_step'],2), d.get('report_ms_per_step'))"
  done
done
unset KSIM_SCAN1_MIX
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_report.py > $OUT/tests2.log 2>&1 || { tail -30 $OUT/tests2.log; exit 1; }
tail -3 $OUT/tests2.log
