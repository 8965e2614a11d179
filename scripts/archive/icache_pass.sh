#!/bin/bash
# instruction-cache counters of the dominant kernel (one --pmc pass per configuration)
export TMPDIR=/tmp KSIM_COOP=0
mkdir -p gpurun_out/ic
for cfg in "c2:" "c2rm5:--run-mode 5" "c5:--config c5 --steps 1 --warmup 0"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/ic/$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $args > gpurun_out/ic/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ic/$name.log; exit 1; }
  python3 - "$name" <<'PY'
import csv, glob, sys
name = sys.argv[1]
acc = {}
for f in glob.glob("gpurun_out/ic/%s/**/*counter_collection.csv" % name, recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(t in k for t in ("k_memo<", "k_hmemo<", "k_replay<")): continue
        acc.setdefault(k[:40], {}).setdefault(r["Counter_Name"], 0.0)
        acc[k[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    req = v.get("SQC_ICACHE_REQ", 0) or 1
    print(name, k, {c: int(x) for c, x in v.items()}, "miss rate %.4f" % (v.get("SQC_ICACHE_MISSES", 0) / req))
PY
done
