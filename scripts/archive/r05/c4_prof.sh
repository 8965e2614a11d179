#!/bin/bash
# r05: C4 group timeline (replay / report ends per group) and a kernel-trace profile of the C4 bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
KSIM_GROUP_TIMES=1 timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1 \
  > $OUT/c4.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
grep "group times" $OUT/c4.err | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 3 --warmup 1 \
  > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
cut -c1-160 $OUT/kernel_stats.csv | head -12
