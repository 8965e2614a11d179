#!/bin/bash
# wide k_hmemo: C5 tests, C5 bench + phase profile
mkdir -p gpurun_out/w
timeout -k 10 200 python3 bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/w/c5.json 2> gpurun_out/w/c5.err || { tail gpurun_out/w/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/w/c5.json'));print('c5', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['wgs_per_replica'])"
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "ksim hmemo profile" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_c5.py \
  > gpurun_out/w/c5t.log 2>&1; rc=$?; grep -E "PASS|FAIL|C5" gpurun_out/w/c5t.log; tail -3 gpurun_out/w/c5t.log; [ $rc = 0 ] || exit 1
