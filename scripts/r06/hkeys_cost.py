"""What the keys in HBM cost a widened FGD chain: gpushare100 (seed 48) at K workgroups on k_memo beside one narrow FGD
replica (the split run of a sweep share), alone in its launch (keys in LDS) and with a gpuspec33 replica (seed 42, 32
workgroups: 42.6 ms alone, shorter) in the same launch (every key in HBM); KSIM_GROUP_TIMES=1 prints each group's end.
Usage: KSIM_GROUP_TIMES=1 python3 scripts/r06/hkeys_cost.py [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim.sweep as SW  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
base = [("openb_pod_list_gpushare100", "06-FGD", 48, 1.3), ("openb_pod_list_gpushare100", "06-FGD", 42, 1.3)]
for name, items, wide in (("lds", base, {0: K}),
                          ("hbm", base + [("openb_pod_list_gpuspec33", "06-FGD", 42, 1.3)], {0: K, 2: 32})):
    sw = SW.Sweep(items, wgs=1, wide=wide)
    ms = min(sw.run()[0] for _ in range(3))
    print(name, K, round(ms, 2), sw.eng.last_run_kernels(), flush=True)
    sw.close()
