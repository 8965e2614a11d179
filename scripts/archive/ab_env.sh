#!/bin/bash
# Interleaved A/B of environment settings on one box: bash scripts/ab_env.sh "A=1" "A=0 B=2" ... (each twice)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for round in 1 2; do
  for envs in "$@"; do
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 ${BENCH_ARGS:-} > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo "bench [$envs] rc=$?"; tail gpurun_out/ab/b.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/b.json'));print(sys.argv[1],'ms/launch %.2f'%d['device_ms_per_step'])" "[$envs]"
  done
done
