#!/bin/bash
# Interleaved A/B of two library builds on one box: bash scripts/r06/ab.sh OUT ROUNDS [bench args...]
# (base = lib/ab/libksim_hip_base.so, new = the in-tree lib/libksim_hip.so); one line per run: label, ms per step.
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
for ((i = 0; i < R; i++)); do
  for v in base new; do
    if [ $v = base ]; then L=kubernetes-scheduler-simulator_amd/lib/ab/libksim_hip_base.so; else L=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so; fi
    KSIM_LIB_PATH=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "$v run $i rc=$?"; exit 1; }
    python3 -c "import json; d = json.load(open('$O/ab_${v}_$i.json')); print('$v', $i, round(d['device_ms_per_step'], 3), round(d['ms_per_step'], 3))"
  done
done
