"""One C4 share (--rank-share k/N's experiments and plan_widths' widened FGD replicas) run whole and by part --
the widened FGD replicas alone (k_memo), the other FGD replicas alone (k_hmemo), the cheap policies alone
(k_scan1_mix) -- device ms (best of 3) and the launched kernels; KSIM_GROUP_TIMES=1 adds each group's end.
Usage: python3 scripts/r06/share_parts.py k/N [wide K] [cheap replicas per CU] [whole]  (no K: plan_widths' choice;
K: every widened replica at K; K 0: none widened)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))
import ksim.sweep as SW  # noqa: E402

k, n = (int(x) for x in sys.argv[1].split("/"))
kw = int(sys.argv[2]) if len(sys.argv) > 2 else None
pc = int(sys.argv[3]) if len(sys.argv) > 3 else 3
only_whole = len(sys.argv) > 4
items = SW.plan()
exps = SW.shard(items, k, n, SW.plan_costs(items))
costs = SW.plan_costs(exps)
wcosts = SW.plan_wide_costs(exps)
if kw is None:
    wide = SW.plan_widths(exps, costs, wcosts, slack=int(os.environ.get("SHARE_SLACK", SW.CU_SLACK)))
elif kw == 0:
    wide = {}
else:
    wide = SW.plan_widths(exps, costs, wcosts, ks=(kw,), packs=((pc, 1.0),))
wc = {i: wcosts[k][i] for i, k in wide.items()}
print(json.dumps({"share": sys.argv[1], "experiments": len(exps), "wide": len(wide), "wide_k": sorted(wide.values()), "per_cu_cheap": pc,
                  "wide_exps": [exps[i][:3] for i in sorted(wide)],
                  "est_ms": {"narrow_fgd_max": max((costs[i] for i, e in enumerate(exps) if e[1] == "06-FGD" and i not in wide),
                                                   default=0) / 1000,
                             "wide_max": max(wc.values(), default=0) / 1000,
                             "cheap_max": max((costs[i] for i, e in enumerate(exps) if e[1] != "06-FGD"), default=0) / 1000}}),
      flush=True)
parts = {"whole": list(range(len(exps))), "wide": sorted(wide),
         "narrow_fgd": [i for i, e in enumerate(exps) if e[1] == "06-FGD" and i not in wide],
         "cheap": [i for i, e in enumerate(exps) if e[1] != "06-FGD"]}
for name, idx in parts.items():
    if not idx or (only_whole and name != "whole"):
        continue
    sub = [exps[i] for i in idx]
    w = {j: wide[i] for j, i in enumerate(idx) if i in wide}
    sw = SW.Sweep(sub, wgs=1, wide=w)
    ms = min(sw.run()[0] for _ in range(3))
    print(json.dumps({"part": name, "experiments": len(sub), "device_ms": round(ms, 2),
                      "kernels": sw.eng.last_run_kernels(), "gate": sw.eng.last_run_gate()}), flush=True)
    sw.close()
