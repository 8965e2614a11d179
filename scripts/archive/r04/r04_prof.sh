#!/bin/bash
# r04 measurement on one box: C2 against the r03 library (interleaved), the counter passes of every headline
# configuration (scripts/profile_all.sh -> gpurun_out/prof/<name>/), one cooperative-launch FETCH_SIZE pass of C2
# beside the plain-launch one (are the counters the same?), and the node-sharded C5 over two shard processes.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r04prof; mkdir -p $O
export TMPDIR=/tmp
R03=KSIM_LIB_PATH=$PWD/abtmp/r03/libksim_hip.so
one() {  # tag bench-args env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err
  local rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag: %.3f ms device %.3f' % (d['ms_per_step'], d['device_ms_per_step']))"
}
for i in 1 2 3; do
  one c2_r03_$i "--steps 10 --warmup 2" $R03
  one c2_r04_$i "--steps 10 --warmup 2"
done
bash scripts/profile_all.sh c2 c2-rm5 c2-PWR_500_FGD_500 c4 c5 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_coop -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_coop.log 2>&1
echo "coop FETCH_SIZE pass rc=$?"
python3 - <<'PY'
import csv, glob
def per_kernel(d):
    out = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "k_memo<" not in k: continue
            out.setdefault(k, []).append(float(row.get("Counter_Value", 0)))
    return {k: (len(v), sum(v) / max(len(v), 1)) for k, v in out.items()}
print("coop  ", per_kernel("gpurun_out/r04prof/fetch_coop"))
import json
d = json.load(open("gpurun_out/prof/c2/pmc.json"))
print("plain ", {k: v for k, v in d.get("dominant", {}).items() if "fetch" in k.lower() or "hbm" in k.lower() or k == "kernel"})
PY
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --config c5 --sharded --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_sharded_world2.json 2> $O/c5_sharded_world2.err
rc=$?; echo "sharded world 2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/c5_sharded_world2.err; exit $rc; }
python3 -c "import json; d=json.loads(open('$O/c5_sharded_world2.json').read().strip().splitlines()[-1]); print('c5 sharded world 2: %.1f ms per 1M-pod replay, %.0f pods/s' % (d['ms_per_step'], d['value']))"
