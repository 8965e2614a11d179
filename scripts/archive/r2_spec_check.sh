#!/bin/bash
mkdir -p gpurun_out/s2
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_memo.py -k "hmemo or deletions or tiny or workgroups" \
  > gpurun_out/s2/memo.log 2>&1; rc=$?; tail -2 gpurun_out/s2/memo.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/s2/memo.log | head; exit 1; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py -k "prefix or step_kernel or full" \
  > gpurun_out/s2/c5.log 2>&1; rc=$?; tail -2 gpurun_out/s2/c5.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/s2/c5.log | head; exit 1; }
timeout -k 10 200 python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s2/c5.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/s2/c5.json'));print('c5', round(d['value']), round(d['ms_per_step'],2))"
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
