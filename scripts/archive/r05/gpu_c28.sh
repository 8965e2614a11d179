#!/bin/bash
# r05: C5 at other workgroup counts per replica (--wgs; auto = 63, S = 1600) on the tree without the wide-form L2
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r05c28}; mkdir -p $OUT
for i in 1 2; do
  for k in ${KS:-0 40 50 80 100}; do
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 --wgs $k > $OUT/c5_k${k}_$i.json 2> $OUT/c5_k${k}_$i.err || { echo "c5 k$k $i failed"; tail -5 $OUT/c5_k${k}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_k${k}_$i.json')); print('c5 wgs $k $i', round(d['ms_per_step'],1), d['config'].get('wgs_per_replica'))" | tee -a $OUT/summary.txt
  done
done
