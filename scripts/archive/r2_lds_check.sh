#!/bin/bash
# k_replay per-policy LDS layout + two K=1 workgroups per CU: parity, report, sweep rows, C4 / C3 timing
mkdir -p gpurun_out/l
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_report.py \
  tests/test_gpu_residency.py tests/test_gpu_sweep.py tests/test_gpu_pwr.py > gpurun_out/l/t.log 2>&1; rc=$?
tail -2 gpurun_out/l/t.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/l/t.log | head -20; exit 1; }
timeout -k 10 200 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/l/c4.json 2>gpurun_out/l/c4.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/l/c4.json'));print('c4', round(d['value']), round(d['ms_per_step'],2), d['experiments_per_s'])"
for pol in BestFit GpuClustering; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --policy $pol > gpurun_out/l/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/l/b.json'));print('$pol', round(d['value']), round(d['ms_per_step'],2))"
done
