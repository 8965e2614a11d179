#!/bin/bash
# r05: C4 counter profile (the cheap k_scan1_mix now bounds it), C5 bench, then the rank-share rehearsal
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c9
bash scripts/profile_config.sh c4 --config c4 || exit 1
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r05c9/c5.json 2> gpurun_out/r05c9/c5.err || { tail -5 gpurun_out/r05c9/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05c9/c5.json')); print('c5', round(d['ms_per_step'],1))"
bash scripts/r05/c4_shares.sh
