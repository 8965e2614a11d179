#!/bin/bash
# KSIM_HPF A/B (k_hmemo at one workgroup per replica): 0 = wave 1 lists, 1 = wave 0 lists the next refresh
# after its Bind, 3 = + touches the next refresh's flagged rows.  Parity with 3 first, then interleaved timings.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/hpf
mkdir -p $O
export TMPDIR=/tmp
KSIM_HPF=3 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_memo.py tests/test_gpu_sweep.py tests/test_gpu_fuzz.py -m gpu > $O/pytest_hpf3.log 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest_hpf3.log; exit 1; }
tail -1 $O/pytest_hpf3.log
j() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3))" "$@"; }
for i in 1 2; do
  for f in 0 1 3; do
    KSIM_HPF=$f timeout -k 10 120 python3 bench.py --run-mode 5 --steps 5 --warmup 1 --no-cpu-baseline > $O/rm5_$f.log 2>&1 || exit 1
    j $O/rm5_$f.log "rm5 hpf=$f"
    KSIM_HPF=$f timeout -k 10 120 python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > $O/c4_$f.log 2>&1 || exit 1
    j $O/c4_$f.log "c4 hpf=$f"
  done
done
KSIM_HPF=3 KSIM_PROFILE=1 timeout -k 10 120 python3 bench.py --run-mode 5 --steps 1 --warmup 0 --no-cpu-baseline > $O/rm5_prof3.log 2>&1 || exit 1
grep "hmemo profile" $O/rm5_prof3.log
