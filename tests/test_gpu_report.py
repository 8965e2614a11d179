"""GPU parity of the per-event cluster report (analysis.go:59-119 ClusterGpuFragReport).

Bar: for every event, the device report equals the oracle's exact-sum report bit for bit (7
cluster bins, used nodes / GPUs / GPU milli / CPU milli, arrived GPU / CPU milli), and its bins
are within 1e-9 relative of the oracle's literal fp64 sum in node order (the reference's sum
order is a Go map's; north_star's curve tolerance).  The [Power] report that follows it
(analysis.go:24-56, with the trace's energy model set on every replica) equals the oracle's per-node
GetEnergyConsumptionNode sums exactly on every event.  Every test needs a gfx950 device.
"""
import pytest

import helpers
import ksim
import ksim.analysis as A
import pyoracle as O

pytestmark = pytest.mark.gpu

POLICIES = [("FGD", O.POL_FGD, O.SEL_FGD), ("BestFit", O.POL_BESTFIT, O.SEL_BEST),
            ("DotProd", O.POL_DOTPROD, O.SEL_BEST), ("GpuPacking", O.POL_PACKING, O.SEL_BEST),
            ("GpuClustering", O.POL_CLUSTERING, O.SEL_BEST), ("Random", O.POL_RANDOM, O.SEL_RANDOM)]
KEYS = ["used_nodes", "used_gpus", "used_gpu_milli", "total_gpus", "arrived_gpu_milli", "used_cpu_milli",
        "arrived_cpu_milli"]


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def engine_reports(trace, nodes, events, n_ev, policy, seed=0, run_mode=0, wgs=0):
    arr, n = trace.typical()
    eng = ksim.Engine(len(nodes), 1, run_mode=run_mode, wgs_per_replica=wgs)
    eng.set_nodes(0, nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, policy, seed=seed)
    eng.set_power_model(0, trace.power_model())
    eng.set_report(True)
    eng.load_events(0, events, n_ev)
    eng.run()
    res, reps, pw = eng.results(0), eng.reports(0), eng.power_reports(0)
    eng.close()
    for r, p in zip(reps, pw):
        r["power"] = p
    return res, reps


def assert_reports(got, want):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g["frag_bins"] == w["frag_bins_exact"], (i, g["frag_bins"], w["frag_bins_exact"])
        for k in KEYS:
            assert g[k] == w[k], (i, k, g[k], w[k])
        for a, b in zip(g["frag_bins"], w["frag_bins"]):
            assert abs(a - b) <= 1e-9 * max(abs(b), 1.0), (i, a, b)
        if "power" in g:
            p = g["power"]
            assert (p["cpu_w"], p["gpu_w"], p["invalid_nodes"]) == (w["power_cpu"], w["power_gpu"], w["power_invalid"]), \
                (i, p, w["power_cpu"], w["power_gpu"])


def subset(trace, rp, step, off=0):
    keep = list(range(off, trace.num_nodes, step))
    onodes = helpers.oracle_subset(trace, rp, keep)
    return keep, helpers.subset_nodes(rp, keep), onodes


@pytest.mark.parametrize("name,pol,sel", POLICIES, ids=[p[0] for p in POLICIES])
def test_report_subset_all_policies(default_trace, name, pol, sel):
    rp = default_trace.replay(seed=42)
    keep, nodes, onodes = subset(default_trace, rp, 7, 3)
    n_ev = 1500
    res, got = engine_reports(default_trace, nodes, rp.events, n_ev, name, seed=11)
    want_res, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                     helpers.oracle_events(default_trace, rp, n_ev), policy=pol, gpu_sel=sel,
                                     seed=11, threads=16, with_report=True)
    assert res == want_res
    assert_reports(got, want)
    assert got[-1]["used_gpu_milli"] > 0 and got[-1]["arrived_gpu_milli"] > got[-1]["used_gpu_milli"]


@pytest.mark.parametrize("run_mode,wgs", [(2, 1), (2, 5), (2, 64), (1, 0), (3, 3), (3, 7), (3, 0)])
def test_report_execution_paths(default_trace, run_mode, wgs):
    # k_replay (2) with any workgroup split, the k_step (hipGraph) path (1) and k_memo (3) record the same report
    rp = default_trace.replay(seed=3)
    keep, nodes, onodes = subset(default_trace, rp, 4)
    n_ev = 1200
    _, got = engine_reports(default_trace, nodes, rp.events, n_ev, "FGD", run_mode=run_mode, wgs=wgs)
    _, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace),
                              helpers.oracle_events(default_trace, rp, n_ev), policy=O.POL_FGD, gpu_sel=O.SEL_FGD,
                              threads=16, with_report=True)
    assert_reports(got, want)


def test_report_with_deletions(default_trace):
    rp = default_trace.replay(seed=9)
    keep, nodes, onodes = subset(default_trace, rp, 9)
    evs, oev = helpers.delete_stream(default_trace, rp, 900, 0.3, seed=1)
    for run_mode in (1, 2, 3):
        res, got = engine_reports(default_trace, nodes, evs, len(evs), "FGD", run_mode=run_mode)
        want_res, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace), oev, policy=O.POL_FGD,
                                         gpu_sel=O.SEL_FGD, threads=16, with_report=True)
        assert res == want_res
        assert_reports(got, want)
    assert any(r[4] == ksim.DELETED and r[0] >= 0 for r in res)


def test_report_multi_replica_ragged(default_trace):
    cfgs = [(42, "FGD", O.POL_FGD, O.SEL_FGD, 900), (43, "BestFit", O.POL_BESTFIT, O.SEL_BEST, 1300),
            (44, "FGD", O.POL_FGD, O.SEL_FGD, 1100)]
    keep = list(range(0, default_trace.num_nodes, 6))
    arr, n = default_trace.typical()
    eng = ksim.Engine(len(keep), len(cfgs))
    eng.set_report(True)
    rps = []
    for r, (seed, name, _, _, n_ev) in enumerate(cfgs):
        rp = default_trace.replay(seed=seed)
        rps.append(rp)
        eng.set_nodes(r, helpers.subset_nodes(rp, keep))
        eng.set_typical(r, arr, n)
        eng.set_policy(r, name)
        eng.load_events(r, rp.events, n_ev)
    eng.run()
    # the report kernels ran: after a sequential replay the report behind it, after concurrent groups the sum
    # of each group's report timed on its own stream
    assert eng.last_report_ms() > 0
    for r, (seed, name, pol, sel, n_ev) in enumerate(cfgs):
        onodes = helpers.oracle_subset(default_trace, rps[r], keep)
        _, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                  helpers.oracle_events(default_trace, rps[r], n_ev), policy=pol, gpu_sel=sel,
                                  threads=16, with_report=True)
        assert_reports(eng.reports(r), want)
    eng.close()


def test_report_full_openb_fgd_curves(default_trace):
    # C2, seed 42: every event's report on 1213 nodes, then the reference's curves
    rp = default_trace.replay(seed=42)
    res, got = engine_reports(default_trace, rp.nodes, rp.events, rp.n, "FGD")
    onodes = helpers.oracle_nodes(default_trace, rp)
    want_res, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                     helpers.oracle_events(default_trace, rp, rp.n), policy=O.POL_FGD,
                                     gpu_sel=O.SEL_FGD, threads=16, with_report=True)
    assert res == want_res
    assert_reports(got, want)
    cg = A.curves(got)
    cw = A.curves([dict(w, frag_bins=w["frag_bins"]) for w in want])  # literal fp64 node-order sums
    assert cg["alloc"] == cw["alloc"]
    for k in cg["frag"]:
        assert abs(cg["frag"][k] - cw["frag"][k]) <= 0.011, k  # 2-decimal printing of 1e-12-close values
    # expected_results/analysis_allo_discrete.csv, 06-FGD @ 130% arrived: 95.27-95.49 over seeds 42-51
    assert 94.5 < cg["alloc"][130] < 96.0


@pytest.mark.parametrize("side", ["1", "3", "6"])
def test_report_concurrent_groups_side_streams(default_trace, monkeypatch, side):
    # six policy groups at one workgroup per replica run concurrently (FGD on k_hmemo, run_mode 5; the cheap
    # policies on k_scan1), each group's report right behind its replay on that group's stream, over one, three
    # (the FGD group alone + two shared) or six side streams: every event's report and result equal the oracle's
    monkeypatch.setenv("KSIM_SIDE_STREAMS", side)
    keep = list(range(4, default_trace.num_nodes, 9))
    arr, n = default_trace.typical()
    cfgs = [(42 + i, name, pol, sel) for i, (name, pol, sel) in enumerate(POLICIES)]
    eng = ksim.Engine(len(keep), len(cfgs), run_mode=5, wgs_per_replica=1)
    rps = []
    try:
        eng.set_report(True)
        for r, (seed, name, _, _) in enumerate(cfgs):
            rp = default_trace.replay(seed=seed)
            rps.append(rp)
            eng.set_nodes(r, helpers.subset_nodes(rp, keep))
            eng.set_typical(r, arr, n)
            eng.set_policy(r, name, seed=seed)
            eng.load_events(r, rp.events, 700)
        eng.run()
        # FGD on k_hmemo and the five cheap policies as one k_scan1_mix launch, concurrently; each group's
        # report timed on its stream
        launches, streams = eng.last_run_launches()
        assert launches == 2 and streams == min(2, int(side))
        assert eng.last_report_ms() > 0
        # the cheap launch waited for every FGD workgroup's start flag, and the gate opened within its bound
        assert eng.last_run_gate() == (1, 0)
        assert eng.last_run_kernels() == ["k_hmemo", "k_scan1_mix"]
        got = [(eng.results(r), eng.reports(r)) for r in range(len(cfgs))]
    finally:
        eng.close()
    for r, (seed, name, pol, sel) in enumerate(cfgs):
        onodes = helpers.oracle_subset(default_trace, rps[r], keep)
        want_res, _, want = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                         helpers.oracle_events(default_trace, rps[r], 700), policy=pol, gpu_sel=sel,
                                         seed=seed, threads=16, with_report=True)
        assert got[r][0] == want_res, name
        assert_reports(got[r][1], want)
