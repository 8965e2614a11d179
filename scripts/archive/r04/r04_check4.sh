#!/bin/bash
# r04: the fma fold in frag_F_quad and the wide form's wave-0 list (KSIM_HPF=5) -- the whole GPU suite, then
# A/Bs against the r03 library on C2 / C2 run_mode 5 / C4 / PWR 500 FGD 500 / C5, and C2's counter passes.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c4; mkdir -p $O
export TMPDIR=/tmp
R03=KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -1; grep -E "FAILED|Error" $O/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one c2_r03_$i "--steps 10 --warmup 2" $R03
  one c2_r04_$i "--steps 10 --warmup 2"
done
for i in 1 2; do
  one rm5_r03_$i "--steps 5 --warmup 1 --run-mode 5" $R03
  one rm5_r04_$i "--steps 5 --warmup 1 --run-mode 5"
  one c4_r03_$i "--config c4 --steps 3 --warmup 1" $R03
  one c4_r04_$i "--config c4 --steps 3 --warmup 1"
  one pf_r03_$i "--steps 5 --warmup 1 --policy PWR_500_FGD_500" $R03
  one pf_r04_$i "--steps 5 --warmup 1 --policy PWR_500_FGD_500"
  one rm2_r03_$i "--steps 5 --warmup 1 --run-mode 2" $R03
  one rm2_r04_$i "--steps 5 --warmup 1 --run-mode 2"
done
one c5_r03 "--config c5 --steps 2 --warmup 1" $R03
one c5_r04 "--config c5 --steps 2 --warmup 1"
one c5_hpf5 "--config c5 --steps 2 --warmup 1" KSIM_HPF=5
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1; grep "hmemo profile" $O/prof_c5.log | cut -c1-900
bash scripts/profile_all.sh c2 || exit 1
