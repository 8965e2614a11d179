"""Run the paper sweep (C4: 17 traces x 6 policies x seeds 42-51, tune 1.3) on the GPU(s) and
write its curves in the format of the reference's experiments/analysis/expected_results:
  <out>/analysis_allo_discrete.csv, <out>/analysis_frag_discrete.csv  (one row per experiment)
  <out>/compare.json   per (trace, policy): max |ours - reference| of the 10-seed mean curves
                       over arrived-GPU % 0..130; per policy: how many experiments reproduce
                       the reference's row exactly; the sweep's timing
Multi-GPU: torchrun --nproc-per-node N scripts/sweep.py; rank k replays its share of a longest-processing-time
split by ksim.sweep's cost model (ksim.sweep.shard with plan_costs: experiments by falling estimated replay time,
each to the least loaded rank; no collective on the data path); each rank writes its own CSV files (suffix
.rank<k>).  The cost model counts each experiment's events from the Go math/rand replay on the host (cached
per process).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"))

import pandas as pd  # noqa: E402

import ksim.sweep as SW  # noqa: E402

EXPECTED = os.path.join(ROOT, "tests", "golden", "expected_results")


def rows_of(curves, kind):
    out = []
    for (t, p, s), c in sorted(curves.items()):
        row = {"workload": t, "sc_policy": p, "tune": 1.3, "seed": s}
        row.update({str(k): v for k, v in sorted(c[kind].items())})
        out.append(row)
    return pd.DataFrame(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep"))
    ap.add_argument("--traces", default="all")
    ap.add_argument("--fgd-batch", type=int, default=0,
                    help="run the FGD experiments as engines of this many replicas (0: one engine for all)")
    ap.add_argument("--pwr", action="store_true",
                    help="also the fork's PWR runs (07-PWR, 08/11/12 PWR+FGD; no expected_results for them)")
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    traces = SW.TRACES if args.traces == "all" else args.traces.split(",")
    policies = tuple(SW.ALL_POLICY_DIRS) if args.pwr else tuple(SW.POLICY_DIRS)
    items = SW.plan(traces=traces, policies=policies)
    exps = SW.shard(items, rank, world, SW.plan_costs(items) if world > 1 else None)
    t0 = time.perf_counter()
    sw = SW.Sweep(exps, device=local, fgd_batch=args.fgd_batch)
    t_setup = time.perf_counter() - t0
    dev_ms, wall = sw.run()
    t1 = time.perf_counter()
    curves = sw.curves()
    t_curves = time.perf_counter() - t1
    sw.close()
    os.makedirs(args.out, exist_ok=True)
    suffix = "" if world == 1 else ".rank%d" % rank
    rows_of(curves, "alloc").to_csv(os.path.join(args.out, "analysis_allo_discrete.csv" + suffix), index=False)
    rows_of(curves, "frag").to_csv(os.path.join(args.out, "analysis_frag_discrete.csv" + suffix), index=False)
    summary = {"experiments": len(exps), "events": sw.total_events, "device_ms": dev_ms, "run_wall_s": wall,
               "setup_s": t_setup, "curves_s": t_curves, "experiments_per_s": len(exps) / wall, "pairs": {}}
    if world == 1:
        worst = {"alloc": 0.0, "frag": 0.0}
        for t in traces:
            for p in SW.POLICY_DIRS:
                d = {}
                for kind, csv in (("alloc", "analysis_allo_discrete.csv"), ("frag", "analysis_frag_discrete.csv")):
                    ours = SW.mean_curve(curves, t, p, kind)
                    ref = SW.expected_mean_curve(os.path.join(EXPECTED, csv), t, p)
                    keys = [k for k in ours if k in ref]
                    dev = max(abs(ours[k] - ref[k]) for k in keys)
                    d[kind] = {"max_abs_dev": round(dev, 3), "at130_ours": round(ours.get(130, float("nan")), 2),
                               "at130_ref": round(ref.get(130, float("nan")), 2), "points": len(keys)}
                    worst[kind] = max(worst[kind], dev)
                summary["pairs"]["%s/%s" % (t, p)] = d
        summary["worst_max_abs_dev"] = worst
        # row for row: every experiment's curve against the reference's row of the same seed
        rows = {}
        for kind, csv in (("alloc", "analysis_allo_discrete.csv"), ("frag", "analysis_frag_discrete.csv")):
            mm = SW.row_mismatches(curves, kind, SW.expected_rows(os.path.join(EXPECTED, csv)))
            for p in SW.POLICY_DIRS:
                sel = {k: v for k, v in mm.items() if k[1] == p}
                rows.setdefault(p, {})[kind] = {
                    "rows": len(sel), "identical": sum(1 for v in sel.values() if not v),
                    "differing": ["%s/%d: %d points from %s" % (k[0], k[2], len(v), v[0])
                                  for k, v in sorted(sel.items()) if v][:20]}
        summary["rows_identical"] = rows
    with open(os.path.join(args.out, "compare.json" + suffix), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: (v if k != "rows_identical" else {p: {kk: vv["identical"] for kk, vv in d.items()} for p, d in v.items()}) for k, v in summary.items() if k != "pairs"}))


if __name__ == "__main__":
    main()
