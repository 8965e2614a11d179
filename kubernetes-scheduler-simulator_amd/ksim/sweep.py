"""The paper sweep (C4): traces x policies x seeds as independent replicas on one GPU.

Seeds reproduce the reference's event streams and node names exactly (Go math/rand,
csrc/go_rand.hpp), so each experiment's curves can be compared row for row with the
reference's expected_results (row_mismatches).

The reference runs each (trace, policy, seed) experiment as its own `simon apply` process,
1020 of them in ~10 h on 256 vCPUs (experiments/README.md:19-27,69-70; run lists in
experiments/run_scripts/expected_run_scripts_0511.sh).  Here every experiment is one replica of
one ksim.Engine: one k_replay launch per policy replays them all, the device computes every
event's cluster report, and the host turns the reports into the allocation / fragmentation
curves of experiments/analysis/merge_*_discrete.py (ksim.analysis).
"""
import json
import os
import time

import numpy as np

import ksim
import ksim.analysis as A

TRACES = ["openb_pod_list_cpu050", "openb_pod_list_cpu100", "openb_pod_list_cpu200", "openb_pod_list_cpu250",
          "openb_pod_list_default", "openb_pod_list_gpushare100", "openb_pod_list_gpushare40",
          "openb_pod_list_gpushare60", "openb_pod_list_gpushare80", "openb_pod_list_gpuspec10",
          "openb_pod_list_gpuspec20", "openb_pod_list_gpuspec25", "openb_pod_list_gpuspec33",
          "openb_pod_list_multigpu20", "openb_pod_list_multigpu30", "openb_pod_list_multigpu40",
          "openb_pod_list_multigpu50"]
# expected_results' sc_policy directories -> (score plugin, gpuSelMethod) (expected_run_scripts_0511.sh)
POLICY_DIRS = {"01-Random": "Random", "02-DotProd": "DotProd", "03-GpuClustering": "GpuClustering",
               "04-GpuPacking": "GpuPacking", "05-BestFit": "BestFit", "06-FGD": "FGD"}
# the fork's power-aware runs (generate_run_scripts.py:31-42; directory = id-policy with '_' for ' ',
# get_dir_name_from_method :54-63).  No expected_results exist for them.
PWR_POLICY_DIRS = {"07-PWR": "PWR", "08-PWR_500_FGD_500": "PWR 500 FGD 500",
                   "11-PWR_100_FGD_900": "PWR 100 FGD 900", "12-PWR_50_FGD_950": "PWR 50 FGD 950"}
ALL_POLICY_DIRS = {**POLICY_DIRS, **PWR_POLICY_DIRS}
SEEDS = list(range(42, 52))


def plan(traces=TRACES, policies=tuple(POLICY_DIRS), seeds=SEEDS, tune=1.3):
    return [(t, p, s, tune) for t in traces for p in policies for s in seeds]


# Cost model of one experiment on one GPU: its events x the per-event latency of its replay chain, read from the
# measured table (profiles/r06/c4_costs.jsonl, scripts/r06/c4_costs.py: every trace and policy alone on the GPU, the
# seed with the most events, the cluster report on) -- FGD on k_hmemo at one workgroup ("one") and on k_memo at K
# workgroups ("wide<K>"), the cheap policies on k_scan1.  Without the table: the r05 constants (FGD ~4.1 us per
# event up to ~64 typical pods, growing with the typical table beyond, 0.8x widened; the cheap policies ~3.3 us).
COST_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                          "profiles", "r06", "c4_costs.jsonl")
FGD_US, FGD_US_PER_TYP, CHEAP_US = 4.1, 0.055, 3.3
# The widths plan_widths chooses from: k_memo workgroups of a widened FGD replica (per replica since r06: the engine
# launches each at its own width), and how tight the cheap replicas pack -- (replicas planned per CU, how much their
# chains slow down packed that tight: share 0/4 at 6 to a CU, its cheap group 32.6 -> 50.9 ms;
# profiles/r06/c4_shares/widths_r06.txt).  The measured costs per width are in the table (gpushare80 alone: 60.7 ms
# on k_hmemo, 56.9 / 54.3 / 48.3 / 46.8 / 44.2 / 41.6 / 41.3 / 39.5 ms at 6 / 8 / 12 / 16 / 24 / 32 / 48 / 64 workgroups).
WIDE_KS = (6, 8, 12, 16, 24, 32, 48, 64)
CHEAP_PACKS = ((3, 1.0), (6, 1.4))
# A chain within WIDEN_MARGIN of the share's predicted time is widened too while CUs last: beside the others on a full
# GPU every chain runs 3-5 % longer than alone, so a narrow chain just under the widened ones ends after them (share
# 1/8 with 9 widened: 51.2 ms; share 0/8 with 12: 48.3; profiles/r06/c4_shares/widths_r06.txt)
WIDEN_MARGIN = 0.9
# CUs the plan leaves unused: the three launches do not pack the device perfectly, and a plan that fills all 256 lost
# the cheap group's residency (its last replicas waited for CUs: share 1/4 69.6 ms, 2/8 63.4); 16 spare restored it
# (54.4 / 46.8 ms), 32 the same (54.4 / 46.5; profiles/r06/c4_shares/slack_r06.txt).  16 for every share predicts
# shorter shares but measured the same (N = 8 45.6-49.3 ms, N = 4 53.3-54.5: summary_r06sh12_slack16_k64.txt)
CU_SLACK = 32
_COSTS = None


def load_costs(path=COST_TABLE):
    """{(trace, policy, form): us per event} from the measured table ({} when absent)."""
    global _COSTS
    if _COSTS is None or path != COST_TABLE:
        out = {}
        if os.path.exists(path):
            with open(path) as f:
                for ln in f:
                    d = json.loads(ln)
                    if d.get("us_per_event"):
                        form = d["form"]
                        if form == "wide":  # the r06 table's first form: one width, in wgs_req
                            form = "wide%d" % d["wgs_req"]
                        if form.startswith("wide") and not d.get("kernels", ["k_memo"])[0].startswith("k_memo"):
                            continue  # no k_memo plan at that width (the engine fell back): not a width to plan
                        out[(d["trace"], d["policy"], form)] = d["us_per_event"]
        if path != COST_TABLE:
            return out
        _COSTS = out
    return _COSTS


def experiment_cost_us(policy_dir, events, n_typical, trace=None, form="one"):
    """Estimated replay time of one experiment (us): its events x the measured per-event latency of its trace and
    policy in that form (load_costs), or the r05 constants."""
    us = load_costs().get((trace, policy_dir, form))
    if us is not None:
        return events * us
    if policy_dir == "06-FGD":
        return events * (FGD_US + FGD_US_PER_TYP * max(0, n_typical - 64)) * (0.8 if form.startswith("wide") else 1.0)
    return events * CHEAP_US


_EVENTS = {}


def plan_costs(items, form="one"):
    """Estimated cost of each (trace, policy, seed, tune) experiment: the replay's event count (the
    reference's own stream, ksim.Trace.replay) x experiment_cost_us's latency."""
    traces = {}
    out = []
    for (t, p, s, tune) in items:
        if t not in traces:
            traces[t] = ksim.Trace.openb(t[len("openb_pod_list_"):] if t.startswith("openb_pod_list_") else t)
        tr = traces[t]
        k = (t, s, tune)
        if k not in _EVENTS:
            _EVENTS[k] = tr.replay(seed=s, tune_ratio=tune, shuffle=True).n
        out.append(experiment_cost_us(p, _EVENTS[k], tr.typical()[1], t, form))
    return out


def plan_widths(items, costs, wide_costs, cus=256, ks=WIDE_KS, packs=CHEAP_PACKS, margin=WIDEN_MARGIN,
                slack=CU_SLACK):
    """Critical-path-aware widths for one share's experiments (run concurrently on one GPU).  The
    share's time is its longest replay chain: the cheap chains (cheap_slow x the longest, for the packing), the FGD
    chains left on k_hmemo at one workgroup, and the widened ones on k_memo at their width.  Each widened replica holds
    its workgroups' CUs, every other FGD replica one (k_memo and k_hmemo fill a CU's registers), the cheap replicas
    per_cu to a CU, `slack` CUs left over.  For each packing, the shortest predicted time T that fits the CUs: every FGD
    chain longer than T
    widened at the fewest workgroups that bring it under T; then the chains within `margin` of T at the fewest
    workgroups that shorten them, longest first, while CUs last.  The packing with the shorter T wins (ties: the
    first).  wide_costs: {K: a cost per item at K workgroups} (plan_wide_costs).
    -> {item index: workgroups} for the widened ones."""
    fgd = sorted((i for i, it in enumerate(items) if it[1] == "06-FGD"), key=lambda i: (-costs[i], i))
    cheap = [i for i, it in enumerate(items) if it[1] != "06-FGD"]
    ks = sorted(k for k in ks if k in wide_costs)
    best = None
    for n, (per_cu, slow) in enumerate(packs):
        budget = cus - slack - len(fgd) - -(-len(cheap) // per_cu)
        floor = max((costs[i] for i in cheap), default=0.0) * slow
        cands = sorted({floor} | {costs[i] for i in fgd} | {wide_costs[k][i] for k in ks for i in fgd})
        for T in cands:
            if T < floor:
                continue
            out, need, ok = {}, 0, True
            for i in fgd:
                if costs[i] <= T:
                    break
                k = next((k for k in ks if wide_costs[k][i] <= T), None)
                if k is None:
                    ok = False
                    break
                out[i] = k
                need += k - 1
            if not ok or need > budget:
                continue
            for i in fgd:
                if costs[i] <= margin * T:
                    break
                k = next((k for k in ks if wide_costs[k][i] < costs[i]), None)
                if i in out or k is None or need + k - 1 > budget:
                    continue
                out[i] = k
                need += k - 1
            if best is None or (T, n) < best[0]:
                best = ((T, n), out)
            break
    return best[1] if best else {}


def plan_wide_costs(items, ks=WIDE_KS):
    """{K: plan_costs(items, "wide<K>")} for every width of `ks`; an FGD experiment whose trace the table holds but
    not at that width (k_memo has no plan for it: gpuspec33's keys at 6 workgroups) costs inf there."""
    table = load_costs()
    out = {}
    for k in ks:
        c = plan_costs(items, "wide%d" % k)
        if table:
            c = [v if it[1] != "06-FGD" or (it[0], it[1], "wide%d" % k) in table else float("inf")
                 for v, it in zip(c, items)]
        out[k] = c
    return out


def shard(items, rank, world, costs=None):
    """Replica-parallel split across ranks (no collective on the data path).  With `costs` (one per item,
    plan_costs): longest processing time first -- items by falling cost, each to the rank with the least
    cost so far (ties to the lower rank) -- so the long FGD replays spread over the ranks and the totals
    balance; each rank keeps its items in plan order.  Without: round robin (items[rank::world])."""
    if costs is None or world <= 1:
        return items[rank::world]
    load = [0.0] * world
    mine = []
    for i in sorted(range(len(items)), key=lambda i: (-costs[i], i)):
        k = min(range(world), key=lambda j: (load[j], j))
        load[k] += costs[i]
        if k == rank:
            mine.append(i)
    return [items[i] for i in sorted(mine)]


class Sweep:
    """All experiments of a plan as replicas on one device: one engine for the persistent-kernel
    policies (k_memo / k_replay) and, when the plan has PWR experiments, one for those (k_step +
    k_step_pwr per pod)."""

    def __init__(self, experiments, device=0, report=True, wgs=0, fgd_batch=0, random_stream="hash", wide=None):
        """random_stream: "hash" (the Random contract) or "go" (the reference's draw
        structure on Go's math/rand stream, k_random_go: ksim_engine_set_go_stream).  wide: {experiment index:
        workgroups} -- FGD experiments to replay on k_memo at that width beside the one-workgroup ones
        (plan_widths; ksim_engine_set_replica_wgs)."""
        wide = wide or {}
        assert random_stream in ("hash", "go")
        self.exps = list(experiments)
        traces = {}
        for (t, _, _, _) in self.exps:
            if t not in traces:
                traces[t] = ksim.Trace.openb(t[len("openb_pod_list_"):] if t.startswith("openb_pod_list_") else t)
        n_nodes = {tr.num_nodes for tr in traces.values()}
        assert len(n_nodes) == 1, "every trace of a sweep must share the node list"
        nn = n_nodes.pop()
        typ = {name: tr.typical() for name, tr in traces.items()}
        pwr = [i for i, e in enumerate(self.exps) if e[1] in PWR_POLICY_DIRS]
        rest = [i for i, e in enumerate(self.exps) if e[1] not in PWR_POLICY_DIRS]
        self.groups = []
        self.total_events = 0
        parts = [rest, pwr]
        if fgd_batch > 0:  # FGD experiments as separate engines of fgd_batch replicas (k_memo where they fit)
            fgd = [i for i in rest if self.exps[i][1] == "06-FGD"]
            fgd_set = set(fgd)
            parts = [[i for i in rest if i not in fgd_set], pwr] + \
                [fgd[k:k + fgd_batch] for k in range(0, len(fgd), fgd_batch)]
        for idx in parts:
            if not idx:
                continue
            eng = ksim.Engine(nn, len(idx), device=device, wgs_per_replica=wgs)
            if report:
                eng.set_report(True)
            for r, i in enumerate(idx):
                t, p, s, tune = self.exps[i]
                rp = traces[t].replay(seed=s, tune_ratio=tune, shuffle=True)
                eng.set_nodes(r, rp.nodes)
                arr, n = typ[t]
                eng.set_typical(r, arr, n)
                eng.set_policy(r, ALL_POLICY_DIRS[p], seed=s)
                if i in wide:
                    eng.set_replica_wgs(r, wide[i])
                # every experiment: PWR's energy model, and the per-event [Power] report the reference
                # logs after every event whatever the policy (simulator.go:427)
                eng.set_power_model(r, traces[t].power_model())
                if p == "01-Random" and random_stream == "go":
                    eng.set_go_stream(r, traces[t].go_state(seed=s, tune_ratio=tune, shuffle=True))
                eng.load_events(r, rp.events, rp.n)
                self.total_events += rp.n
            self.groups.append((eng, idx))
        self.eng = self.groups[0][0]  # the persistent-kernel engine (bench.py --config c4)
        self.report = report

    def fgd_replicas(self, group=0):
        """Replica indices of one group's engine that run FGD (the memoised paths)."""
        return [r for r, i in enumerate(self.groups[group][1]) if self.exps[i][1] == "06-FGD"]

    def run(self):
        t0 = time.perf_counter()
        dev_ms = sum(eng.run() for eng, _ in self.groups)
        return dev_ms, time.perf_counter() - t0

    def curves(self):
        """{(trace, policy, seed): {"alloc": {arr%: val}, "frag": ..., "frag_ratio": ...}}"""
        assert self.report
        out = {}
        for eng, idx in self.groups:
            for r, i in enumerate(idx):
                t, p, s, _ = self.exps[i]
                out[(t, p, s)] = A.curves_arrays(eng.report_arrays(r))
        return out

    def close(self):
        for eng, _ in self.groups:
            eng.close()


def mean_curve(curves, trace, policy, kind="alloc"):
    """Mean over seeds of one (trace, policy) curve: {arrived %: mean}."""
    rows = [c[kind] for (t, p, _), c in curves.items() if t == trace and p == policy]
    keys = sorted(set.intersection(*[set(r) for r in rows]))
    return {k: float(np.mean([r[k] for r in rows])) for k in keys}


def expected_rows(csv_path):
    """expected_results/analysis_*_discrete.csv -> {(trace, policy, seed): {arrived %: value}}"""
    import pandas as pd
    df = pd.read_csv(csv_path)
    cols = [c for c in df.columns if c.isdigit()]
    out = {}
    for rec in df.to_dict(orient="records"):
        out[(rec["workload"], rec["sc_policy"], int(rec["seed"]))] = {
            int(c): float(rec[c]) for c in cols if rec[c] == rec[c]}  # NaN: no data at that %
    return out


def row_mismatches(curves, kind, expected):
    """Per experiment: the arrived-GPU % at which our curve differs from the reference's row
    (values compared exactly: both are 2-decimal roundings of the same computation)."""
    out = {}
    for key, c in curves.items():
        ref = expected.get(key)
        if ref is None:
            continue
        ours = c[kind]
        out[key] = sorted(k for k in set(ours) | set(ref) if ours.get(k) != ref.get(k))
    return out


def max_rel_dev(ours, ref):
    """Largest relative deviation |ours - ref| / |ref| over the points both curves have (absolute where
    ref is 0); +inf when the point sets differ."""
    if set(ours) != set(ref):
        return float("inf")
    return max((abs(ours[k] - ref[k]) / abs(ref[k]) if ref[k] else abs(ours[k])) for k in ref) if ref else 0.0


def expected_mean_curve(csv_path, trace, policy, seeds=SEEDS):
    """The reference's expected_results/analysis_*_discrete.csv mean over seeds."""
    import pandas as pd
    df = pd.read_csv(csv_path)
    df = df[(df.workload == trace) & (df.sc_policy == policy) & (df.seed.isin(list(seeds)))]
    cols = [c for c in df.columns if c.isdigit()]
    return {int(c): float(df[c].mean()) for c in cols if df[c].notna().all()}
