#!/bin/bash
# k_scan1 with the node records in VGPRs (KSIM_SCAN1=2) against LDS (1): parity, then C4 timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/reg; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sweep.py -k "single_workgroup or full_paper" -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
for r in 1 2; do for m in 1 2; do
  KSIM_SCAN1=$m timeout -k 10 300 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > $O/b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('c4 KSIM_SCAN1=$m dev ms %.2f'%d['device_ms_per_step'], flush=True)"
done; done
for m in 2 1; do KSIM_SCAN1=$m timeout -k 10 300 python3 scripts/c4_groups.py > $O/c4g_$m.log 2>&1; echo "KSIM_SCAN1=$m $(tail -1 $O/c4g_$m.log)"; done
