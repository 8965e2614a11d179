"""k_hmemo's phase split (KSIM_PROFILE=1, the general instantiation) on one C4 FGD trace at a time:
10 seeds at one workgroup per replica.  Usage: KSIM_PROFILE=1 python3 scripts/r05/hmemo_phases.py TRACE..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim.sweep as SW  # noqa: E402

for t in sys.argv[1:]:
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_" + t], policies=["06-FGD"]), report=False)
    ms = sw.run()[0]
    print("trace", t, "device ms", round(ms, 2), "events", max(sw.eng.n_events), flush=True)
    sw.close()
