#!/bin/bash
# Interleaved A/B of prebuilt libraries over several bench configurations on one box.
# Usage: bash scripts/ab_configs.sh "bench args 1;bench args 2" a.so b.so ...   (each pair run twice)
# Prints device ms per launch for each (config, library); restores the in-tree library at the end.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $LIB gpurun_out/ab/orig.so.bak
IFS=';' read -ra CFGS <<< "$1"
shift
for round in 1 2; do
  for cfg in "${CFGS[@]}"; do
    for so in "$@"; do
      cp "$so" $LIB
      timeout -k 10 300 python bench.py --no-cpu-baseline $cfg > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err \
        || { echo "bench [$cfg] $so rc=$?"; tail gpurun_out/ab/b.err; cp gpurun_out/ab/orig.so.bak $LIB; exit 1; }
      python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/b.json'));print('[%s] %s dev ms %.2f'%(sys.argv[2],sys.argv[1],d['device_ms_per_step']),flush=True)" "$so" "$cfg"
    done
  done
done
cp gpurun_out/ab/orig.so.bak $LIB
