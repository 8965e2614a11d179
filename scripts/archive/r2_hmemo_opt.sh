#!/bin/bash
# k_hmemo changes: parity (memo -k hmemo, fuzz FGD paths, c5 prefix), then timing + phase profiles
mkdir -p gpurun_out/h
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_memo.py -k "hmemo" \
  > gpurun_out/h/memo.log 2>&1; rc=$?; tail -2 gpurun_out/h/memo.log; [ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/h/memo.log | head; exit 1; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -k "FGD" \
  > gpurun_out/h/fuzz.log 2>&1; rc=$?; tail -2 gpurun_out/h/fuzz.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c5.py -k "prefix or step_kernel" \
  > gpurun_out/h/c5.log 2>&1; rc=$?; tail -2 gpurun_out/h/c5.log; [ $rc = 0 ] || exit 1
for a in "--config c5 --steps 1 --warmup 1" "--run-mode 5" "--config c4"; do
  timeout -k 10 200 python3 bench.py $a --no-cpu-baseline > gpurun_out/h/b.json 2> gpurun_out/h/b.err || { tail gpurun_out/h/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/h/b.json'));print('$a', round(d['value']), round(d['ms_per_step'],2), d['roofline']['kernel'], d['roofline']['wgs_per_replica'])"
done
for a in "--config c5 --steps 1 --warmup 0" "--run-mode 5 --steps 1 --warmup 0"; do
  KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py $a --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
done
