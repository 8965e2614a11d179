"""What the in-kernel report records (snap / prev per event) cost a replay chain: one paper-sweep experiment alone,
FGD on k_hmemo (one workgroup) and on k_memo at K workgroups, BestFit on k_scan1, with and without the report;
device ms (best of 3).  Usage: python3 scripts/r06/report_cost.py trace:seed ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim  # noqa: E402


def engine(tr, seed, pol, wgs, run_mode, report):
    eng = ksim.Engine(tr.num_nodes, 1, wgs_per_replica=wgs, run_mode=run_mode)
    eng.set_report(report)
    rp = tr.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    eng.set_nodes(0, rp.nodes)
    arr, n = tr.typical()
    eng.set_typical(0, arr, n)
    eng.set_policy(0, pol, seed=seed)
    eng.set_power_model(0, tr.power_model())
    eng.load_events(0, rp.events, rp.n)
    return eng, rp.n


for arg in sys.argv[1:]:
    t, _, s = arg.partition(":")
    tr = ksim.Trace.openb(t)
    for pol, wgs, mode in (("FGD", 1, 5), ("FGD", 16, 3), ("BestFit", 1, 0)):
        for rep in (False, True):
            eng, n = engine(tr, int(s), pol, wgs, mode, rep)
            try:
                ms = min(eng.run() for _ in range(3))
                out = {"device_ms": round(ms, 3), "us_per_event": round(ms * 1000 / n, 3), "path": eng.last_run_path(),
                       "kernels": eng.last_run_kernels(), "report_ms": round(eng.last_report_ms(), 3) if rep else 0}
            except ksim.KsimError as ex:
                out = {"error": str(ex)}
            eng.close()
            print(json.dumps({"trace": t, "seed": int(s), "policy": pol, "wgs": wgs, "report": rep, "events": n, **out}),
                  flush=True)
