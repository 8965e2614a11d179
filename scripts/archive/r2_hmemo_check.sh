set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_memo.py tests/test_gpu_fuzz.py -k "hmemo or (all_paths and FGD) or (cluster_report and FGD)" -p no:cacheprovider > $O/memo.log 2>&1 || { echo "memo tests rc=$?"; tail -30 $O/memo.log; exit 1; }
tail -3 $O/memo.log
KSIM_PROFILE=1 timeout -k 10 300 python bench.py --run-mode 5 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_h_prof.json 2> $O/bench_h_prof.err || { echo "prof rc=$?"; tail $O/bench_h_prof.err; exit 1; }
grep hmemo $O/bench_h_prof.err | head -3
timeout -k 10 300 python bench.py --run-mode 5 --steps 5 --no-cpu-baseline > $O/bench_h.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > $O/bench_m.json 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c4 --steps 2 > $O/bench_c4.json 2>&1 || exit 1
python3 -c "
import json
for f in ['bench_h','bench_m','bench_c4']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['roofline']['kernel'], 'dev ms %.2f'%d['device_ms_per_step'], 'value %.3g'%d['value'])
"
