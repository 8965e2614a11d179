"""C4's FGD group trace by trace: 10 seeds of one trace on k_hmemo (one workgroup per replica), device ms
per run (best of 3), events, typical pods (T) and score groups, to see which traces bound the group.
Usage: python3 scripts/c4_fgd_traces.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim  # noqa: E402
import ksim.sweep as SW  # noqa: E402

traces = sorted({e[0] for e in SW.plan()})
for t in traces:
    sw = SW.Sweep(SW.plan(traces=[t], policies=["06-FGD"]))
    ms = min(sw.run()[0] for _ in range(3))
    ev = max(sw.eng.n_events)
    sw.close()
    tr = ksim.Trace.openb(t[len("openb_pod_list_"):])
    _, nt = tr.typical()
    print(json.dumps({"trace": t, "device_ms": round(ms, 2), "max_events": ev, "typical": nt,
                      "us_per_step": round(ms * 1000 / max(ev, 1), 3)}), flush=True)
