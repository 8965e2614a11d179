#!/bin/bash
# Timing of the replay under different engine configurations + one rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"FGD:0:0 FGD:8:0 FGD:16:0 FGD:25:0 FGD:0:1 BestFit:0:0"}
for v in $VARIANTS; do
  IFS=: read pol wgs mode <<< "$v"
  timeout -k 10 300 python bench.py --policy $pol --wgs $wgs --run-mode $mode --steps 3 --warmup 1 --no-cpu-baseline \
     > gpurun_out/bench_${pol}_${wgs}_${mode}.log 2>&1 || { echo "bench $v failed rc=$?"; tail -5 gpurun_out/bench_${pol}_${wgs}_${mode}.log; exit 1; }
  tail -1 gpurun_out/bench_${pol}_${wgs}_${mode}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), 'pods/s', round(d['device_ms_per_step'],1),'ms/step', 'wgs', d['roofline'].get('wgs_per_replica'))"
  grep "ksim profile" gpurun_out/bench_${pol}_${wgs}_${mode}.log | tail -1 || true
done
if [ "${PROF:-1}" = "1" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fgd -o fgd --output-format csv -- \
   python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_fgd.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
cat gpurun_out/prof_fgd/fgd_kernel_stats.csv
fi
