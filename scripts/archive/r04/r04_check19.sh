#!/bin/bash
# r04: C4 as the final-tree suite runs it (the CPU baseline's 16 worker processes first) against --no-cpu-baseline,
# interleaved: is the ~178 ms mode tied to the baseline's process pool?
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c19; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one c4_cpu_$i "--config c4"
  one c4_nocpu_$i "--config c4 --no-cpu-baseline"
done
