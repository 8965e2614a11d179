#!/bin/bash
# r04: the one-runtime process on a GPU box -- smoke, the runtime maps after real device work, the new
# stress / peer tests, the C2 bench, and ONE cooperative-launch FETCH_SIZE counter pass (verdict r03 item 2).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04rt
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139) return 0;; *) return 1;; esac; }
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/r04rt/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/r04rt/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step maps 200 python -u -c "
import sys, json; sys.path[:0] = ['kubernetes-scheduler-simulator_amd', '.']
import ksim, bench
t = ksim.Trace.openb('default'); eng = bench._engine_on(0, t, [42, 43], 0); eng.run()
import torch; torch.cuda.set_device(0); torch.cuda.synchronize(); x = torch.ones(4, device='cuda'); print(float(x.sum()))
eng.run(); eng.close(); print(json.dumps(ksim.hip_runtimes()))"
step memotests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_memo.py
step newtests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_hdelay.py tests/test_gpu_shard.py -k "hdelay or delay or peer or device_exchange"
step bench 300 python -u bench.py
step pmc_coop 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r04rt/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
find gpurun_out/r04rt/fetch -name "*.csv" | head -5
