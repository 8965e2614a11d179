#!/bin/bash
# A/B of k_hmemo's batched F (default) against one quad per item (KSIM_HBATCH=0), interleaved on one box:
# C2 run_mode 5 (ten one-workgroup replicas), C4 (the sweep's FGD group), C5 (the wide form); then the
# KSIM_PROFILE=1 phase split of run_mode 5 for both.  Usage: bash scripts/hbatch_ab.sh [configs...]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/hbatch
out=gpurun_out/hbatch/ab.txt
: > $out
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("--run-mode 5" "--config c4" "--config c5")
for i in 1 2; do
  for hb in 1 0; do
    for cfg in "${cfgs[@]}"; do
      r=$(KSIM_HBATCH=$hb timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $cfg 2>/dev/null | tail -1) || { echo "bench failed: $cfg"; exit 1; }
      echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('HBATCH=$hb', '$cfg'.ljust(14), 'kernel %-14s' % d['roofline']['kernel'], 'ms/step %.2f' % d['ms_per_step'], 'dev ms %.2f' % d['device_ms_per_step'], 'us/pod-step %.3f' % d['latency']['us_per_pod_step'])" | tee -a $out
    done
  done
done
for hb in 1 0; do
  KSIM_HBATCH=$hb KSIM_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --run-mode 5 2>&1 | grep "ksim hmemo" | sed "s/^/HBATCH=$hb /" | tee -a $out
done
