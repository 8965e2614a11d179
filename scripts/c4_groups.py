"""C4 sweep: each policy group alone and all together (device ms per run, best of 3), to see how the
concurrent groups share the GPU.  Usage: python3 scripts/c4_groups.py [policy dirs...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim.sweep as SW  # noqa: E402

out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
groups = [(p,) for p in (sys.argv[1:] or SW.POLICY_DIRS)] + [tuple(SW.POLICY_DIRS)]
for pols in groups:
    sw = SW.Sweep(SW.plan(policies=pols), report=True)
    ms = min(sw.run()[0] for _ in range(3))
    sw.close()
    out["+".join(pols) if len(pols) < 6 else "all"] = round(ms, 2)
    print(json.dumps(out), flush=True)
