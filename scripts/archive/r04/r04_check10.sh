#!/bin/bash
# r04: C4's run-to-run spread (133-149 ms on most runs, ~180 on some): the default against k_hmemo asking for
# a whole CU's LDS (KSIM_HMEMO_EXCL=1: no other group's workgroup beside a k_hmemo one) and against three side
# streams (FGD alone + two for the five short groups), interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c10; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3 4; do
  one c4_def_$i "--config c4 --steps 3 --warmup 1"
  one c4_excl_$i "--config c4 --steps 3 --warmup 1" KSIM_HMEMO_EXCL=1
  [ $i -le 2 ] && one c4_s3_$i "--config c4 --steps 3 --warmup 1" KSIM_SIDE_STREAMS=3
done
exit 0
