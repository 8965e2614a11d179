#!/bin/bash
# A/B of the dead-class skip: C4 (k_hmemo + k_scan1 groups) and C5 (wide k_hmemo), interleaved
mkdir -p gpurun_out
for i in 1 2; do
  for s in 1 0; do
    KSIM_SKIP=$s timeout -k 10 200 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab4_$s.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab4_$s.log') if l.startswith('{')][-1]); print('c4 skip=$s', round(d['ms_per_step'],3))"
  done
done
for s in 1 0; do
  KSIM_SKIP=$s timeout -k 10 200 python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab5_$s.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab5_$s.log') if l.startswith('{')][-1]); print('c5 skip=$s', round(d['ms_per_step'],3))"
done
