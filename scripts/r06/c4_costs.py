"""The sweep's cost table (ksim.sweep.load_costs): for every trace and policy of the paper sweep, the seed with the
most events replayed alone on the GPU with the cluster report, in the form a sweep share gives it -- one workgroup
(FGD on k_hmemo, the cheap policies on k_scan1) -- and, for FGD, k_memo at each wide width (form "wide<K>"); device
ms (best of 3) and us per event.  One JSON line per (trace, policy, form).
Usage: python3 scripts/r06/c4_costs.py [wide K,K,..., default 16,12] > profiles/r06/c4_costs.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim  # noqa: E402
import ksim.sweep as SW  # noqa: E402

KWS = [int(k) for k in (sys.argv[1] if len(sys.argv) > 1 else "16,12").split(",")]
for t in SW.TRACES:
    tr = ksim.Trace.openb(t[len("openb_pod_list_"):])
    ev = {s: tr.replay(seed=s, tune_ratio=1.3, shuffle=True).n for s in SW.SEEDS}
    seed = max(ev, key=ev.get)
    for pol in SW.POLICY_DIRS:
        for wgs in ([1] + KWS if pol == "06-FGD" else [1]):
            sw = SW.Sweep([(t, pol, seed, 1.3)], report=True, wgs=1, wide={0: wgs} if wgs > 1 else None)
            try:
                ms = min(sw.eng.run() for _ in range(3))
                out = {"device_ms": round(ms, 3), "us_per_event": round(ms * 1000 / ev[seed], 4),
                       "kernels": sw.eng.last_run_kernels(), "wgs": sw.eng.last_run_wgs()}
            except ksim.KsimError as ex:
                out = {"error": str(ex)}
            sw.close()
            print(json.dumps({"trace": t, "policy": pol, "seed": seed, "events": ev[seed], "form": "wide%d" % wgs if wgs > 1 else "one",
                              "wgs_req": wgs, **out}), flush=True)
