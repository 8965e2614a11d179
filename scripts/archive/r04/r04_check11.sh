#!/bin/bash
# r04: C4 with the FGD group's stream at the greatest priority (default now) against all streams at the default
# priority (KSIM_SIDE_PRIO=0), and with k_hmemo asking for a whole CU (KSIM_HMEMO_EXCL=1, which made the slow
# placement common in r04c10) under both; interleaved.  Then the sweep's parity once.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c11; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3 4; do
  one c4_prio_$i "--config c4 --steps 3 --warmup 1"
  one c4_noprio_$i "--config c4 --steps 3 --warmup 1" KSIM_SIDE_PRIO=0
  one c4_excl_prio_$i "--config c4 --steps 3 --warmup 1" KSIM_HMEMO_EXCL=1
  one c4_excl_noprio_$i "--config c4 --steps 3 --warmup 1" KSIM_HMEMO_EXCL=1 KSIM_SIDE_PRIO=0
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_sweep.py tests/test_gpu_report.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; exit $rc
