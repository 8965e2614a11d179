#!/bin/bash
# r05 final-tree check on one box: the whole GPU suite, smoke, the C2 / C4 / C5 bench lines (bench.py's defaults:
# C2 and C4 with their CPU baselines first)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05suite}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -v --durations=30 --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" $OUT/pytest_gpu.log | tail -2
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -5 $OUT/bench_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -5 $OUT/bench_c5.err; exit 1; }
for c in c2 c4 c5; do python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['ms_per_step'],2), '%.4g' % d['value'], d['unit'], (d.get('cpu_baseline') or {}).get('value'))"; done
