#!/bin/bash
# r05: k_hmemo F-list group pruning -- memo / sweep / hdelay parity, phase split with and without, C4 A/B,
# then the rank-share rehearsal
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c7; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_sweep.py tests/test_gpu_hdelay.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 64 100000; do
  KSIM_HPRUNE=$v KSIM_PROFILE=1 timeout -k 10 300 python -u scripts/r05/hmemo_phases.py default gpuspec10 gpuspec33 > $OUT/phases_$v.log 2>&1 || { tail -5 $OUT/phases_$v.log; exit 1; }
  echo "== KSIM_HPRUNE=$v"; grep -E "^trace|hmemo profile" $OUT/phases_$v.log | cut -c1-400
done
bash scripts/r05/c4_ab.sh r05c7 2 "prune:KSIM_HPRUNE=64" "noprune:KSIM_HPRUNE=100000"
