#!/bin/bash
# k_hmemo after the dead-set double buffer: parity (KSIM_HPF=1), then C4 x10 sweeps and run_mode 5 per
# KSIM_HPF mode, interleaved; a bounded bulk wait that times out prints its state.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/hdiag
mkdir -p $O
export TMPDIR=/tmp
KSIM_HPF=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_memo.py tests/test_gpu_sweep.py tests/test_gpu_c5.py -m gpu > $O/pytest_hpf1.log 2>&1 || { echo "pytest rc=$?"; grep -E "timeout|FAIL|Error" $O/pytest_hpf1.log | head; tail -5 $O/pytest_hpf1.log; exit 1; }
tail -1 $O/pytest_hpf1.log
j() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3))" "$@"; }
for i in 1; do
  for f in 0 1 3; do
    KSIM_HPF=$f timeout -k 10 200 python3 bench.py --config c4 --steps 10 --warmup 1 --no-cpu-baseline > $O/c4_$f.log 2>&1 || { echo "c4 hpf=$f rc=$?"; grep timeout $O/c4_$f.log | head -3; exit 1; }
    j $O/c4_$f.log "c4 hpf=$f"
    KSIM_HPF=$f timeout -k 10 120 python3 bench.py --run-mode 5 --steps 5 --warmup 1 --no-cpu-baseline > $O/rm5_$f.log 2>&1 || { echo "rm5 hpf=$f rc=$?"; exit 1; }
    j $O/rm5_$f.log "rm5 hpf=$f"
  done
done
