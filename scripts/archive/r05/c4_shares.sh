#!/bin/bash
# r05: the 1-GPU rehearsal of the N-GPU C4 strong-scaling run -- every rank's share of the LPT split at
# N = 2, 4, 8 timed alone on this GPU (bench.py --rank-share k/N); the max over k predicts the N-GPU time
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r05c6}; mkdir -p $OUT
for N in 2 4 8; do
  for k in $(seq 0 $((N-1))); do
    KSIM_GROUP_TIMES=1 timeout -k 10 240 python -u bench.py --config c4 --rank-share $k/$N --no-cpu-baseline --steps 5 --warmup 1 \
      > $OUT/share_${k}of${N}.json 2> $OUT/share_${k}of${N}.err || { echo "share $k/$N failed"; tail -5 $OUT/share_${k}of${N}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/share_${k}of${N}.json')); print('$k/$N', d['config']['replicas_per_gpu'], round(d['ms_per_step'],2))" | tee -a $OUT/summary.txt
  done
done
