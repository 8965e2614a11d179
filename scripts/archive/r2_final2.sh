#!/bin/bash
# Round-end evidence after the lean k_hmemo: re-profile the k_hmemo configurations, the C4 / C5 bench
# lines, the whole GPU suite, smoke(), the default bench line.
set -o pipefail
export TMPDIR=/tmp
bash scripts/r2_refresh_profiles.sh c2-rm5 c5 c4 || exit 1
mkdir -p gpurun_out/suite
timeout -k 10 900 python3 -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider tests > gpurun_out/suite/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/suite/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/suite/pytest_gpu.log | head
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/suite/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/suite/bench.json 2> gpurun_out/suite/bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/suite/bench.json'));print('c2', d['value'], d['ms_per_step'])"
