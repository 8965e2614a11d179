#!/bin/bash
# C3: every policy at C2's workload (10 seeds of openb default, one GPU), one line each
mkdir -p gpurun_out/c3
for pol in FGD BestFit DotProd GpuPacking GpuClustering Random PWR "PWR 500 FGD 500" BestFit DotProd; do
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --policy "$pol" > gpurun_out/c3/b.json 2>gpurun_out/c3/b.err || { tail gpurun_out/c3/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c3/b.json'));print('%-16s %10.0f pods/s %7.2f ms %s' % ('$pol', d['value'], d['ms_per_step'], d['roofline']['kernel']))" | tee -a gpurun_out/c3/summary.txt
done
