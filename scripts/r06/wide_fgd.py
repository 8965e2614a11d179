"""One paper-sweep FGD experiment alone on k_memo at K workgroups (run_mode 3: the keys in LDS when they fit, else
in HBM) with the cluster report, against the sweep's one-workgroup k_hmemo form: device ms (best of 3), and whether
every result and report equals the k_hmemo run's.
Usage: python3 scripts/r06/wide_fgd.py trace[:K,K,...] ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim  # noqa: E402
import ksim.sweep as SW  # noqa: E402


def engine(tr, seed, wgs, run_mode):
    eng = ksim.Engine(tr.num_nodes, 1, wgs_per_replica=wgs, run_mode=run_mode)
    eng.set_report(True)
    rp = tr.replay(seed=seed, tune_ratio=1.3, shuffle=True)
    eng.set_nodes(0, rp.nodes)
    arr, n = tr.typical()
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD", seed=seed)
    eng.set_power_model(0, tr.power_model())
    eng.load_events(0, rp.events, rp.n)
    return eng, rp.n


for arg in sys.argv[1:]:
    t, _, ks = arg.partition(":")
    ks = [int(k) for k in ks.split(",")] if ks else [25, 32, 64]
    tr = ksim.Trace.openb(t)
    ev = {s: tr.replay(seed=s, tune_ratio=1.3, shuffle=True).n for s in SW.SEEDS}
    seed = max(ev, key=ev.get)
    base, n = engine(tr, seed, 1, 5)
    ms = min(base.run() for _ in range(3))
    want = (base.results(0), base.reports(0))
    print(json.dumps({"trace": t, "seed": seed, "events": n, "form": "k_hmemo K=1", "device_ms": round(ms, 3),
                      "us_per_event": round(ms * 1000 / n, 3)}), flush=True)
    base.close()
    for k in ks:
        eng, _ = engine(tr, seed, k, 3)
        try:
            ms = min(eng.run() for _ in range(3))
            same = (eng.results(0), eng.reports(0)) == want
            out = {"form": "k_memo", "path": eng.last_run_path(), "wgs": eng.last_run_wgs(),
                   "device_ms": round(ms, 3), "us_per_event": round(ms * 1000 / n, 3), "equal_to_hmemo": same}
        except ksim.KsimError as ex:
            out = {"form": "k_memo", "wgs": k, "error": str(ex)}
        eng.close()
        print(json.dumps({"trace": t, "seed": seed, "events": n, **out}), flush=True)
