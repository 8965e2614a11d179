#!/bin/bash
# C3: the bench line of every policy at C2's workload (10 seeds of openb default, one GPU), then C4.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/c3
mkdir -p $OUT
export TMPDIR=/tmp
for pol in FGD BestFit DotProd GpuPacking GpuClustering Random; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --policy $pol > $OUT/bench_$pol.json 2> $OUT/bench_$pol.err || { echo "bench $pol rc=$?"; tail $OUT/bench_$pol.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],'%.0f pods/s'%d['value'],'%.2f ms/launch'%d['device_ms_per_step'],d['roofline']['kernel'])" $OUT/bench_$pol.json $pol
done
timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 rc=$?"; tail $OUT/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c4.json'));print('C4',d['value'],d['unit'],d['device_ms_per_step'])"
