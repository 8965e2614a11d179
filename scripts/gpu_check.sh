#!/bin/bash
# Runs the GPU checks in order on a gpurun box; every GPU step has its own time
# limit, and a crash/timeout (124, 137, 134, 139) ends the script immediately.
# An ordinary test failure (exit 1) is recorded and the next step still runs.
# Usage: bash scripts/gpu_check.sh [smoke|tests|bench|prof]...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|-6|-11) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    testsall) run pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
