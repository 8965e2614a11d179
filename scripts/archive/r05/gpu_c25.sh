#!/bin/bash
# r05: C5 (wide k_hmemo, K = 63) under the existing knobs, interleaved on one box: the default, KSIM_HL2=0 (no
# per-(class, block) second maxima), KSIM_HPF=5 (the binding workgroup's wave 0 lists the next refresh), KSIM_HPF=0,
# and the r03 library (abtmp_r03)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c25; mkdir -p $OUT
for i in 1 2; do
  for spec in "def:" "hl2off:KSIM_HL2=0" "hpf5:KSIM_HPF=5" "hpf0:KSIM_HPF=0" "r03:KSIM_LIB_PATH=$PWD/abtmp_r03/libksim_hip.so"; do
    label=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_${label}_$i.json 2> $OUT/c5_${label}_$i.err || { echo "c5 $label $i failed"; tail -5 $OUT/c5_${label}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_${label}_$i.json')); print('c5 $label $i', round(d['ms_per_step'],1))" | tee -a $OUT/summary.txt
  done
done
