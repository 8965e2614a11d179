#!/bin/bash
# k_memo A/B on a gpurun box: the memo parity tests, then the default bench line (no CPU leg).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_memo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/memo_tests.log 2>&1 || { echo "memo tests rc=$?"; tail -30 $OUT/memo_tests.log; exit 1; }
tail -2 $OUT/memo_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('ms/launch',d['device_ms_per_step'],'pods/s',d['value'])"
