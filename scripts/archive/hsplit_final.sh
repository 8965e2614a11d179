#!/bin/bash
# After the k_hmemo critical/bulk split: C4 x10 sweeps, the C5 / run_mode 5 lines, then counter profiles.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/hsplit
export TMPDIR=/tmp
O=gpurun_out/hsplit
j() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3), d['roofline']['kernel'])" "$@"; }
echo "c4 $(date +%T)"
timeout -k 10 120 python3 bench.py --config c4 --steps 10 --warmup 1 --no-cpu-baseline > $O/c4_10.log 2>&1 || { echo "c4 rc=$?"; tail -5 $O/c4_10.log; exit 1; }
j $O/c4_10.log c4
echo "rm5 $(date +%T)"
timeout -k 10 120 python3 bench.py --run-mode 5 --steps 10 --warmup 1 --no-cpu-baseline > $O/rm5_10.log 2>&1 || { echo "rm5 rc=$?"; exit 1; }
j $O/rm5_10.log c2-rm5
echo "c5 $(date +%T)"
timeout -k 10 200 python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_2.log 2>&1 || { echo "c5 rc=$?"; exit 1; }
j $O/c5_2.log c5
echo "profiles $(date +%T)"
bash scripts/profile_all.sh c2-rm5 c4 c5
