#!/bin/bash
# r05 C4 A/B on one box, interleaved: bash scripts/r05/c4_ab.sh OUTDIR ROUNDS "label:VAR=VAL,VAR=VAL" ...
# (label "cpu:..." runs bench.py's default order, the CPU baseline's worker pool first)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; ROUNDS=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    extra="--no-cpu-baseline"; case $label in cpu*) extra="";; esac
    envargs=$(echo "$envs" | tr ',' ' ')
    env $envargs KSIM_GROUP_TIMES=1 timeout -k 10 300 python -u bench.py --config c4 $extra --steps 5 --warmup 1 \
      > $OUT/c4_${label}_$i.json 2> $OUT/c4_${label}_$i.err || { echo "bench $label $i failed"; tail -5 $OUT/c4_${label}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_${label}_$i.json')); print('$label', $i, round(d['ms_per_step'],2), round(d['device_ms_per_step'],2), round(d.get('report_ms_per_step') or 0, 2))" | tee -a $OUT/summary.txt
  done
done
