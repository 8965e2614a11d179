#!/bin/bash
# bench.py's N-GPU path with two ranks on a one-GPU box (gloo for the barrier and the job reduction, each rank its
# own seeds on the one device; small engines so both ranks' persistent kernels are resident at once).
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --replicas 2 --wgs 4 --steps 3 --warmup 1 --no-cpu-baseline \
  > $O/c2_world2.json 2> $O/c2_world2.err || { echo "world 2 rc=$?"; tail -20 $O/c2_world2.err; exit 1; }
cat $O/c2_world2.json
