#!/bin/bash
# k_replay workgroups-per-replica sweep for the non-FGD policies at C2 (one GPU).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wgsp
for pol in BestFit GpuPacking; do
  for w in 25 1 2 4 8 25 1; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 3 --policy $pol --wgs $w > gpurun_out/wgsp/$pol.$w.json 2> gpurun_out/wgsp/$pol.$w.err || { echo "$pol wgs $w rc=$?"; tail -5 gpurun_out/wgsp/$pol.$w.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],'wgs',sys.argv[3],d['roofline']['kernel'],d['roofline']['wgs_per_replica'],'ms %.2f'%d['device_ms_per_step'])" gpurun_out/wgsp/$pol.$w.json $pol $w
  done
done
