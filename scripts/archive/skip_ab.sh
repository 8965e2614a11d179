#!/bin/bash
# A/B of the dead-class skip on the C2 bench (interleaved, device ms per launch)
mkdir -p gpurun_out
for i in 1 2 3; do
  for s in 1 0; do
    KSIM_SKIP=$s timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$s.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$s.log') if l.startswith('{')][-1]); print('skip=$s', round(d['ms_per_step'],3), round(d['device_ms_per_step'],3))"
  done
done
