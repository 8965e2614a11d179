#!/bin/bash
# r05: k_scan1_mix with 32-bit argmax keys + the branch-free Filter, against the previous library (abtmp_prev)
# and against the same library with 64-bit keys (KSIM_SCAN1_K32=0) -- parity first, then C4 interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c20; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_scan1_mix.py tests/test_gpu_dotprod.py tests/test_gpu_sweep.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_shard.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/r05/c4_ab.sh r05c20 3 "k32:KSIM_SCAN1_K32=1" "k64:KSIM_SCAN1_K32=0" "prev:KSIM_LIB_PATH=$PWD/abtmp_prev/libksim_hip.so"
