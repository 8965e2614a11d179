#!/bin/bash
# Interleaved A/B of prebuilt libraries on one box: bash scripts/ab_bench.sh a.so b.so ... (each run twice)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $LIB gpurun_out/ab/orig.so.bak
for round in 1 2; do
  for so in "$@"; do
    cp "$so" $LIB
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo "bench $so rc=$?"; tail gpurun_out/ab/b.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/b.json'));print(sys.argv[1],'ms/launch %.2f'%d['device_ms_per_step'])" "$so"
  done
done
cp gpurun_out/ab/orig.so.bak $LIB
