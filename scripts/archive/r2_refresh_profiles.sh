#!/bin/bash
# Re-profile the configurations whose kernels changed, put the summaries where bench.py reads them,
# then the bench lines of C4 and C5 (with their CPU baselines).
set -o pipefail
export TMPDIR=/tmp
for n in "$@"; do
  bash scripts/profile_all.sh $n || exit 1
  mkdir -p profiles/r02/prof/$n && cp gpurun_out/prof/$n/pmc.json gpurun_out/prof/$n/kernel_stats.csv profiles/r02/prof/$n/
done
timeout -k 10 400 python3 bench.py --config c4 --steps 3 > gpurun_out/prof/bench_c4.json 2> gpurun_out/prof/bench_c4.err || { tail gpurun_out/prof/bench_c4.err; exit 1; }
timeout -k 10 400 python3 bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/prof/bench_c5.json 2> gpurun_out/prof/bench_c5.err || { tail gpurun_out/prof/bench_c5.err; exit 1; }
python3 -c "
import json
for f in ['bench_c4','bench_c5']:
    d=json.load(open('gpurun_out/prof/'+f+'.json')); print(f, round(d['value']), 'ms %.2f'%d['ms_per_step'], d['roofline']['kernel'], d['roofline'].get('traffic'))
"
