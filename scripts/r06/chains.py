"""The longest single-replica chains of the paper sweep (C4), one experiment alone on the GPU, in every form
the engine has: FGD on k_hmemo at one workgroup (the sweep's form), k_memo at K workgroups; the cheap
policies on k_scan1 (one workgroup) and k_replay at K workgroups.  With the cluster report (the sweep's
setting).  Prints one JSON line per (experiment, form): device ms (best of 3), events, us per event.
Usage: python3 scripts/r06/chains.py [trace ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim  # noqa: E402
import ksim.sweep as SW  # noqa: E402

traces = sys.argv[1:] or ["openb_pod_list_gpushare100", "openb_pod_list_gpuspec33"]
forms = {"06-FGD": [(1, 0), (0, 3), (25, 3), (16, 3), (8, 3), (4, 3)],
         "05-BestFit": [(1, 0), (2, 2), (4, 2), (8, 2), (16, 2), (25, 2)],
         "04-GpuPacking": [(1, 0), (4, 2), (16, 2)]}
for t in traces:
    tr = ksim.Trace.openb(t[len("openb_pod_list_"):])
    ev = {s: tr.replay(seed=s, tune_ratio=1.3, shuffle=True).n for s in SW.SEEDS}
    seed = max(ev, key=ev.get)
    for pol, fl in forms.items():
        for wgs, rm in fl:
            for report in (True, False) if pol == "06-FGD" and wgs != 1 else (True,):
                sw = SW.Sweep([(t, pol, seed, 1.3)], report=report, wgs=wgs)
                if rm:
                    sw.groups[0][0].close()
                    eng = ksim.Engine(tr.num_nodes, 1, wgs_per_replica=wgs, run_mode=rm)
                    if report:
                        eng.set_report(True)
                    rp = tr.replay(seed=seed, tune_ratio=1.3, shuffle=True)
                    eng.set_nodes(0, rp.nodes)
                    arr, n = tr.typical()
                    eng.set_typical(0, arr, n)
                    eng.set_policy(0, SW.ALL_POLICY_DIRS[pol], seed=seed)
                    eng.set_power_model(0, tr.power_model())
                    eng.load_events(0, rp.events, rp.n)
                else:
                    eng = sw.eng
                try:
                    ms = min(eng.run() for _ in range(3))
                    path, k = eng.last_run_path(), eng.last_run_wgs()
                except ksim.KsimError as ex:
                    ms, path, k = None, str(ex), wgs
                print(json.dumps({"trace": t, "policy": pol, "seed": seed, "events": ev[seed], "wgs_req": wgs,
                                  "run_mode": rm, "report": report, "path": path, "wgs": k,
                                  "device_ms": ms and round(ms, 3),
                                  "us_per_event": ms and round(ms * 1000 / ev[seed], 3)}), flush=True)
                eng.close()
