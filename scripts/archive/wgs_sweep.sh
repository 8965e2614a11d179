set -u
mkdir -p gpurun_out/wgs
for w in 25 20 17 22 25 20; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 3 --wgs $w > gpurun_out/wgs/b$w.json 2> gpurun_out/wgs/b$w.err || { echo "wgs $w rc=$?"; tail -5 gpurun_out/wgs/b$w.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('wgs',sys.argv[2],d['roofline']['kernel'],d['roofline']['wgs_per_replica'],'ms %.2f'%d['device_ms_per_step'])" gpurun_out/wgs/b$w.json $w
done
