#!/bin/bash
# A/B of the dead-class skip on k_replay policies (C3 lines)
mkdir -p gpurun_out
for pol in BestFit PWR; do
  for s in 1 0; do
    KSIM_SKIP=$s timeout -k 10 200 python3 bench.py --policy $pol --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab3_$s.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab3_$s.log') if l.startswith('{')][-1]); print('$pol skip=$s', round(d['ms_per_step'],3), d['roofline']['kernel'])"
  done
done
