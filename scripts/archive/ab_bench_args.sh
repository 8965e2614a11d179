#!/bin/bash
# Interleaved A/B of prebuilt libraries for several bench argument sets:
#   bash scripts/ab_bench_args.sh "a.so b.so" "--policy BestFit" "--config c4" ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
LIB=kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
cp $LIB gpurun_out/ab/orig.so.bak
LIBS=$1; shift
for args in "$@"; do
  for round in 1 2; do
    for so in $LIBS; do
      cp "$so" $LIB
      timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo "bench $so [$args] rc=$?"; tail gpurun_out/ab/b.err; cp gpurun_out/ab/orig.so.bak $LIB; exit 1; }
      python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/b.json'));print(sys.argv[1],sys.argv[2],'ms/launch %.2f'%d['device_ms_per_step'])" "$so" "[$args]"
    done
  done
done
cp gpurun_out/ab/orig.so.bak $LIB
