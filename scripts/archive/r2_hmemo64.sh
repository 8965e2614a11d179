#!/bin/bash
mkdir -p gpurun_out/m
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_memo.py -k hmemo tests/test_gpu_sweep.py \
  > gpurun_out/m/t.log 2>&1; rc=$?; tail -2 gpurun_out/m/t.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/m/t.log | head; exit 1; }
for a in "--config c4" "--run-mode 5" "--config c4"; do
  timeout -k 10 200 python3 bench.py $a --no-cpu-baseline > gpurun_out/m/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/m/b.json'));print('$a', round(d['value']), round(d['ms_per_step'],2))"
done
