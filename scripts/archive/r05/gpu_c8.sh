#!/bin/bash
# r05: k_hmemo per-model tables -- parity (memo, sweep incl. the 850 rows, hdelay, fuzz), phase split and
# per-trace FGD timings with and without (KSIM_HMODEL=0), C4 A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c8; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_sweep.py tests/test_gpu_hdelay.py tests/test_gpu_fuzz.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 1 0; do
  KSIM_HMODEL=$v KSIM_PROFILE=1 timeout -k 10 300 python -u scripts/r05/hmemo_phases.py gpuspec10 gpuspec33 > $OUT/phases_$v.log 2>&1 || { tail -5 $OUT/phases_$v.log; exit 1; }
  echo "== KSIM_HMODEL=$v"; grep -E "^trace" $OUT/phases_$v.log; grep -o "bulk: F (F waves) [0-9.]*\|critical own-class refresh [0-9.]*" $OUT/phases_$v.log
done
timeout -k 10 400 python -u scripts/c4_fgd_traces.py > $OUT/c4_fgd_traces.jsonl 2> $OUT/c4_fgd_traces.err || { tail -5 $OUT/c4_fgd_traces.err; exit 1; }
grep gpuspec $OUT/c4_fgd_traces.jsonl
bash scripts/r05/c4_ab.sh r05c8 2 "model:KSIM_HMODEL=1" "nomodel:KSIM_HMODEL=0"
