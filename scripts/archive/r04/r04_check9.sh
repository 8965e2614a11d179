#!/bin/bash
# r04: k_replay<PWR+FGD> with the per-(class, slot) memo in LDS -- parity (every PWR GPU test, the memo
# off and across its version wrap), then C2 "PWR 500 FGD 500" with and without it, interleaved, and the
# memo's phase profile.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pwr.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  one pf_memo_$i "--policy PWR_500_FGD_500 --steps 5 --warmup 1"
  one pf_nomemo_$i "--policy PWR_500_FGD_500 --steps 5 --warmup 1" KSIM_PF_MEMO=0
done
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --policy PWR_500_FGD_500 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_pf.log 2>&1; grep -o "ksim profile.*" $O/prof_pf.log
