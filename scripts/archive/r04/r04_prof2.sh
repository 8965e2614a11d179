#!/bin/bash
# r04 final-kernel counter passes (scripts/profile_all.sh -> gpurun_out/prof/<name>/) of the configurations whose
# kernels changed after profiles/r04/prof/c2 (k_hmemo: C4, C5, run_mode 5; k_replay<PWR+FGD>), then C5 node-sharded
# over two shard processes on the one GPU.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04prof2; mkdir -p $O
export TMPDIR=/tmp
bash scripts/profile_all.sh c2-rm5 c2-PWR_500_FGD_500 c4 c5 || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --config c5 --sharded --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_sharded_world2.json 2> $O/c5_sharded_world2.err
rc=$?; echo "sharded world 2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/c5_sharded_world2.err; exit $rc; }
python3 -c "import json; d=json.loads(open('$O/c5_sharded_world2.json').read().strip().splitlines()[-1]); print('c5 sharded world 2: %.1f ms per 1M-pod replay, %.0f pods/s' % (d['ms_per_step'], d['value']))"
