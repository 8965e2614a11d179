#!/bin/bash
# Prefetch variant A/B, then the whole GPU suite and smoke() with it in place.
set -o pipefail
export TMPDIR=/tmp
bash scripts/r2_hmemo_ab.sh abtmp/head.so abtmp/pf.so || exit 1
cp abtmp/pf.so kubernetes-scheduler-simulator_amd/lib/libksim_hip.so
mkdir -p gpurun_out/suite
timeout -k 10 900 python3 -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider tests > gpurun_out/suite/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/suite/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/suite/pytest_gpu.log | head
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/suite/smoke.log; exit $rc
