#!/bin/bash
# Kernel-level timing of the step kernel under different policies / block sizes (rocprofv3 kernel trace).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "FGD 32" "FGD 16" "FGD 64" "BestFit 32"; do
  set -- $v
  timeout -k 10 300 python bench.py --policy $1 --nodes-per-block $2 --steps 3 --warmup 1 --no-cpu-baseline \
     > gpurun_out/bench_$1_$2.log 2>&1 || { echo "bench $v failed rc=$?"; exit 1; }
  tail -1 gpurun_out/bench_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), 'pods/s', round(d['roofline']['kernel_us'],2), 'us/kern', round(d['device_ms_per_step'],1),'ms/step')"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fgd -o fgd --output-format csv -- \
   python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_fgd.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
find gpurun_out/prof_fgd -name "*stats*" | head
