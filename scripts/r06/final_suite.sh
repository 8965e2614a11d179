#!/bin/bash
# The round's final evidence on one gpurun box: the whole GPU suite, smoke(), and the default bench line of c2 / c4 /
# c5 (with their CPU baselines); everything under gpurun_out/$1/.  Usage: bash scripts/r06/final_suite.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=30 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
cat $O/smoke.log
for c in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json; d = json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['unit'], round(d['ms_per_step'], 3), d.get('cpu_baseline', {}).get('value'))"
done
