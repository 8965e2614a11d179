#!/bin/bash
# r04 final-tree checks on one box: smoke, the whole GPU suite (with durations), the default bench line and
# the C4 / C5 bench lines.  Every step has its own limit; a crash or a timeout ends the script.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04suite; mkdir -p $O
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139) return 0;; *) return 1;; esac; }
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --durations=40 --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
step bench_c2 300 python -u bench.py
step bench_c4 300 python -u bench.py --config c4
step bench_c5 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline
