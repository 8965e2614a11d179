#!/bin/bash
# k_hmemo critical/bulk split: the k_hmemo parity tests, then C2 run_mode 5 / C4 / C5 timings and one
# KSIM_PROFILE=1 phase print.  Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/hsplit
export TMPDIR=/tmp
O=gpurun_out/hsplit
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_memo.py tests/test_gpu_c5.py tests/test_gpu_fuzz.py tests/test_gpu_shard.py tests/test_gpu_residency.py \
  -m gpu > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sweep.py -m gpu > $O/pytest_sweep.log 2>&1 || { echo "sweep rc=$?"; tail -30 $O/pytest_sweep.log; exit 1; }
tail -2 $O/pytest_sweep.log
j() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3), d['roofline']['kernel'])" "$@"; }
timeout -k 10 200 python3 bench.py --run-mode 5 --steps 5 --warmup 1 --no-cpu-baseline > $O/rm5.log 2>&1 || exit $?
j $O/rm5.log c2-rm5
KSIM_PROFILE=1 timeout -k 10 200 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline > $O/rm5_prof.log 2>&1 || exit $?
grep "hmemo profile" $O/rm5_prof.log | head -2
timeout -k 10 200 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1 || exit $?
j $O/c4.log c4
timeout -k 10 300 python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
j $O/c5.log c5
KSIM_PROFILE=1 timeout -k 10 300 python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/c5_prof.log 2>&1 || exit $?
grep "hmemo profile" $O/c5_prof.log | head -2
