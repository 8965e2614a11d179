#!/bin/bash
# r05: phase profiles (KSIM_PROFILE=1, general instantiations) of C2 PWR 500 FGD 500 (k_replay<PWR+FGD>) and C5 (wide k_hmemo)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c14; mkdir -p $OUT
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --policy "PWR 500 FGD 500" --no-cpu-baseline --steps 1 --warmup 0 > $OUT/pf.json 2> $OUT/pf.err || { tail -5 $OUT/pf.err; exit 1; }
grep -v amdgpu.ids $OUT/pf.err | cut -c1-600 | head -20
KSIM_PROFILE=1 timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 0 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
grep -v amdgpu.ids $OUT/c5.err | cut -c1-900 | head -20
