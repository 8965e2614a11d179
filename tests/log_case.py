"""The log-contract case: one openb run written as `simon apply`'s log, from the oracle or the GPU.

A 243-node subset of the openb GPU nodes (every 5th) under the first 3000 events of openb default
(seed 42, tune 1.3): enough load that pods fail, so the log carries every line kind the reference's
harness reads -- the per-event "[Report]" / "[Alloc]" / "[AllocCPU]" / "[Power]" lines, the
attempt / failure lines, "Failed Pods in detail", the "Cluster Analysis Results (InitSchedule)"
block and "there are N unscheduled pods".  tests/golden/make_log_golden.py runs the reference's own
scripts/analysis.py on the oracle's log (here, where /root/reference exists) and commits what it
produced; tests/test_log_contract.py (CPU) and tests/test_gpu_log_contract.py (GPU) rebuild the log
and compare.
"""
import ksim
import ksim.analysis as A

import helpers

TRACE, SEED, TUNE, STRIDE, N_EVENTS = "default", 42, 1.3, 5, 3000
POLICIES = {"FGD": ("POL_FGD", "SEL_FGD"), "PWR": ("POL_PWR", "SEL_PWR")}


def inputs():
    t = ksim.Trace.openb(TRACE)
    rp = t.replay(seed=SEED, tune_ratio=TUNE, shuffle=True)
    keep = list(range(0, t.num_nodes, STRIDE))
    return t, rp, keep


def pod_lines(t, rp, n):
    """Per event: the pod key (namespace/name; tuned clones "<name>-tuned-<i>", simulator.go:1269) and
    the PodResource fields of its Repr."""
    pods = t.pods()
    n_orig = t.num_pods
    names, reprs = [], []
    for k in range(n):
        p = pods[rp.pod_index[k]]
        name = p["name"] if k < n_orig else "%s-tuned-%d" % (p["name"], k - n_orig)
        names.append("%s/%s" % (A.NAMESPACE, name))
        spec = "|".join(x for x in p["spec"].split("|") if x) if p["num"] > 0 else ""
        reprs.append((p["cpu"], p["milli"] if p["num"] > 0 else 0, p["num"], spec))
    return names, reprs, n_orig


def oracle_log(path, policy):
    """The log of the oracle's run (string-typed restatement, oracle/fgd_oracle.c)."""
    import pyoracle as O
    t, rp, keep = inputs()
    nodes = helpers.oracle_subset(t, rp, keep)
    pol, sel = POLICIES[policy]
    ev = helpers.oracle_events(t, rp, N_EVENTS)
    res, state, reps = O.run_events(nodes, helpers.oracle_typical(t), ev, policy=getattr(O, pol),
                                    gpu_sel=getattr(O, sel), with_report=True)
    final = [dict(cpu_alloc=nd["cpu"], cpu_used=nd["cpu"] - st[0], mem_alloc_mib=nd["mem"],
                  mem_used_mib=nd["mem"] - st[1], gpu_count=nd["gpu"],
                  gpu_used=[1000 - g if j < nd["gpu"] else 0 for j, g in enumerate(st[3])])
             for nd, st in zip(nodes, state)]
    reports = [dict(r, frag_bins=r["frag_bins_exact"]) for r in reps]
    power = [dict(cpu_w=r["power_cpu"], gpu_w=r["power_gpu"]) for r in reps]
    assert all(r["power_invalid"] == 0 for r in reps)
    names, reprs, n_orig = pod_lines(t, rp, len(ev))
    A.write_log(path, reports, pod_names=names, power=power, pods=reprs, results=[r[4] for r in res],
                final_nodes=final, n_original=n_orig)
    return res


def engine_final_nodes(eng, r=0):
    out = []
    for n in eng.nodes(r):
        out.append(dict(cpu_alloc=n.cpu_alloc_milli, cpu_used=n.cpu_used_milli, mem_alloc_mib=n.mem_alloc_mib,
                        mem_used_mib=n.mem_used_mib, gpu_count=n.gpu_count, gpu_used=list(n.gpu_used_milli)))
    return out


def engine_log(path, policy):
    """The log of the GPU engine's run (device reports, device power reports, final state)."""
    t, rp, keep = inputs()
    nodes = helpers.subset_nodes(rp, keep)
    arr, n = t.typical()
    eng = ksim.Engine(len(keep), 1)
    try:
        eng.set_report(True)
        eng.set_nodes(0, nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, policy)
        eng.set_power_model(0, t.power_model())
        eng.load_events(0, rp.events, N_EVENTS)
        eng.run()
        res = eng.results(0)
        reports, power = eng.reports(0), eng.power_reports(0)
        assert all(p["invalid_nodes"] == 0 for p in power)
        names, reprs, n_orig = pod_lines(t, rp, N_EVENTS)
        A.write_log(path, reports, pod_names=names, power=power, pods=reprs, results=[r[4] for r in res],
                    final_nodes=engine_final_nodes(eng), n_original=n_orig)
        return res, eng.last_run_path()
    finally:
        eng.close()
