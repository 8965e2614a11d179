#!/bin/bash
# bench.py's N-GPU path with N ranks on a one-GPU box (gloo for the barrier and the job reduction, each rank its
# own seeds on the one device; small engines so every rank's persistent kernels are resident at once).
# Usage: bash scripts/r06/dist_rehearsal.sh OUTDIR [N, default 2]
set -o pipefail
O=gpurun_out/$1; N=${2:-2}; mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus $N --replicas 2 --wgs 4 --steps 3 --warmup 1 --no-cpu-baseline \
  > $O/c2_world$N.json 2> $O/c2_world$N.err || { echo "world $N rc=$?"; tail -20 $O/c2_world$N.err; exit 1; }
cat $O/c2_world$N.json
