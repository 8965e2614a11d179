#!/bin/bash
mkdir -p gpurun_out/d
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dotprod.py \
  > gpurun_out/d/t.log 2>&1; rc=$?; tail -3 gpurun_out/d/t.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/d/t.log | head -20; exit 1; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
  > gpurun_out/d/p.log 2>&1; rc=$?; tail -2 gpurun_out/d/p.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/d/p.log | head -20; exit 1; }
for pol in DotProd BestFit; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --policy $pol > gpurun_out/d/b.json 2>gpurun_out/d/b.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/d/b.json'));print('$pol', round(d['value']), round(d['ms_per_step'],2))"
done
