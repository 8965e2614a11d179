#!/bin/bash
# C3: the bench line of every policy at C2's workload (10 seeds of openb default, one GPU), then the C4
# and C5 lines.  Each run has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/c3
mkdir -p $OUT
export TMPDIR=/tmp
one() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name rc=$?"; tail $OUT/bench_$name.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],'%.0f %s'%(d['value'],d['unit']),'%.2f ms/launch'%d['device_ms_per_step'],d['roofline']['kernel'])" $OUT/bench_$name.json $name
}
for pol in FGD BestFit DotProd GpuPacking GpuClustering Random PWR PWR_500_FGD_500; do one $pol --policy $pol; done
one fgd_rm2 --run-mode 2
one c4 --config c4
one c5 --config c5 --steps 2 --warmup 1
# node-sharded C5: in-process shard groups (first 5000 events), one shard process, two on the one GPU
timeout -k 10 300 python3 scripts/c5_shard_latency.py > $OUT/c5_shard_inproc.json 2> $OUT/c5_shard_inproc.err || { echo "shard latency rc=$?"; tail $OUT/c5_shard_inproc.err; exit 1; }
tail -c 600 $OUT/c5_shard_inproc.json; echo
one c5_sharded_world1 --config c5 --sharded --steps 1 --warmup 1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --config c5 --sharded --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_sharded_world2_one_gpu.json 2> $OUT/c5w2.err || { echo "c5 world2 rc=$?"; tail $OUT/c5w2.err; exit 1; }
grep '^{' $OUT/bench_c5_sharded_world2_one_gpu.json | cut -c1-200
