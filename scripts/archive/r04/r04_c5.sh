#!/bin/bash
# r04 C5 on one box: the unsharded wide k_hmemo (L2 on / off, interleaved), and the node-sharded mode
# over two shard processes on the one GPU (gloo for the launcher's barrier, device-to-device granules).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04c5; mkdir -p $O
export TMPDIR=/tmp
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.1f ms device %.1f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2; do
  one c5_l2_$i "--config c5 --steps 2 --warmup 1"
  one c5_nol2_$i "--config c5 --steps 2 --warmup 1" KSIM_HL2=0
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --config c5 --sharded --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_sharded_world2.json 2> $O/c5_sharded_world2.err
rc=$?; echo "sharded world 2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/c5_sharded_world2.err; exit $rc; }
python3 -c "import json; d=json.loads(open('$O/c5_sharded_world2.json').read().strip().splitlines()[-1]); print('c5 sharded world 2: %.1f ms per 1M-pod replay, %.0f pods/s' % (d['ms_per_step'], d['value']))"
KSIM_PROFILE=1 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/prof_c5.log 2>&1; grep "hmemo profile" $O/prof_c5.log
