#!/bin/bash
# r05: k_hmemo's residency-gate store moved from the kernel entry into the body (VGPR spills 57 -> 8 at one
# workgroup per replica, 20 -> 11 wide) -- k_hmemo parity (memo forms, C5, hand-over stress, the report / gate,
# the sweep's 850 rows), then C5, C4 and C2 run_mode 5 against the tree before (abtmp_bis/cur2), interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c30; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py tests/test_gpu_c5.py tests/test_gpu_hdelay.py tests/test_gpu_report.py tests/test_gpu_sweep.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for v in new cur2; do
    unset KSIM_LIB_PATH
    [ $v = cur2 ] && export KSIM_LIB_PATH=$PWD/abtmp_bis/cur2/libksim_hip.so
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { echo "c5 $v $i failed"; tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1 > $OUT/c4_${v}_$i.json 2> $OUT/c4_${v}_$i.err || { echo "c4 $v $i failed"; tail -5 $OUT/c4_${v}_$i.err; exit 1; }
    timeout -k 10 300 python -u bench.py --run-mode 5 --no-cpu-baseline --steps 5 --warmup 1 > $OUT/rm5_${v}_$i.json 2> $OUT/rm5_${v}_$i.err || { echo "rm5 $v $i failed"; tail -5 $OUT/rm5_${v}_$i.err; exit 1; }
    python3 -c "
import json
r = [json.load(open('$OUT/%s_${v}_$i.json' % c))['ms_per_step'] for c in ('c5', 'c4', 'rm5')]
print('$v $i c5 %.1f c4 %.2f rm5 %.2f' % tuple(r))" | tee -a $OUT/summary.txt
  done
done
