#!/bin/bash
# The N-GPU C4 rehearsal on one GPU: every share of N = 2, 4, 8 timed alone (bench.py --rank-share k/N), then the
# whole sweep (N = 1); lines under gpurun_out/$1/.  Usage: bash scripts/r06/shares.sh OUTDIR [bench args...]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for N in 8 4 2; do
  for ((k = 0; k < N; k++)); do
    timeout -k 10 120 python3 -u bench.py --config c4 --rank-share $k/$N --no-cpu-baseline --steps 3 --warmup 1 "$@" \
      > $O/share_${k}of${N}.json 2> $O/share_${k}of${N}.err || { echo "share $k/$N rc=$?"; tail -5 $O/share_${k}of${N}.err; exit 1; }
    python3 -c "import json; d = json.load(open('$O/share_${k}of${N}.json')); print('$k/$N', d['config']['replicas_per_gpu'], d['config'].get('widened_fgd'), d['config'].get('wide_k'), round(d['ms_per_step'], 2), d['roofline']['kernel'], d.get('residency_gate'))"
  done
done
