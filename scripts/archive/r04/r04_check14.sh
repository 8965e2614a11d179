#!/bin/bash
# r04: PWR 500 FGD 500 with the memo at fewer workgroups per replica (the memo leaves each workgroup little to
# evaluate, so the exchange's width may matter more): K = 25 (auto) / 20 / 16 / 12, interleaved.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c14; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  for k in 25 20 16 12; do one pf_k${k}_$i "--policy PWR_500_FGD_500 --wgs $k --steps 5 --warmup 1"; done
done
