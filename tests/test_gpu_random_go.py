"""The Random policy's draw structure on Go's math/rand stream (k_random_go, ksim_engine_set_go_stream)
against the oracle's restatement (fgd_oracle.c, orc_policy.go_stream), bit-exact: every event's node,
GPU mask, score, feasible count and status, and the per-event cluster report.

The source state is the stream as the replay driver leaves it (ksim_trace_replay_go_state; pinned
to rand.Seed + the replay's draw count in tests/test_go_rand.py).  The reference's own Random runs
are not reproducible (16 filter workers order its feasible list by timing), so the allocation
curves are compared with expected_results statistically (test_go_stream_sweep_near_expected).
Every test needs a gfx950 device.
"""
import os

import pytest

import helpers
import ksim
import ksim.sweep as SW
import pyoracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ALLO = os.path.join(HERE, "golden", "expected_results", "analysis_allo_discrete.csv")
FRAG = os.path.join(HERE, "golden", "expected_results", "analysis_frag_discrete.csv")
SEL = {"random": O.SEL_RANDOM, "best": O.SEL_BEST, "worst": O.SEL_WORST}


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def run_engine(trace, nodes, events, n_ev, states, gpusel="random", report=False, extra_hash=False):
    arr, n = trace.typical()
    R = len(states) + (1 if extra_hash else 0)
    eng = ksim.Engine(len(nodes), R)
    for r in range(R):
        eng.set_nodes(r, nodes)
        eng.set_typical(r, arr, n)
        eng.set_policy(r, "Random", gpusel=gpusel, seed=5)
        if r < len(states):
            eng.set_go_stream(r, states[r])
        eng.load_events(r, events, n_ev)
    if report:
        eng.set_report(True)
    eng.run()
    out = [eng.results(r) for r in range(R)]
    reps = [eng.reports(r) for r in range(R)] if report else None
    final = [[(x.cpu_used_milli, x.mem_used_mib, x.pods_used, list(x.gpu_used_milli)) for x in eng.nodes(r)]
             for r in range(R)]
    eng.close()
    return out, reps, final


def oracle(trace, rp, keep, n_ev, state, gpusel="random", report=False, events=None):
    onodes = helpers.oracle_subset(trace, rp, keep)
    oev = events if events is not None else helpers.oracle_events(trace, rp, n_ev)
    return O.run_events(onodes, helpers.oracle_typical(trace), oev, policy=O.POL_RANDOM, gpu_sel=SEL[gpusel],
                        seed=5, threads=8, with_report=report, go_stream=state[:3])


@pytest.mark.parametrize("seed", [42, 47])
def test_full_trace_vs_oracle(default_trace, seed):
    # C2's cluster and event stream (all 1213 nodes), Random + random GPU selector
    rp = default_trace.replay(seed=seed)
    st = default_trace.go_state(seed=seed)
    got, _, _ = run_engine(default_trace, rp.nodes, rp.events, rp.n, [st])
    want, _, _ = oracle(default_trace, rp, list(range(default_trace.num_nodes)), rp.n, st)
    assert got[0] == want
    # the draw structure matters: not the hash contract's decisions
    assert sum(1 for r in want if r[0] >= 0) > rp.n // 2


@pytest.mark.parametrize("gpusel", ["random", "best", "worst"])
def test_selectors_and_mixed_engine(default_trace, gpusel):
    # three Go-stream replicas (different seeds' streams) beside a hash-contract Random replica in one
    # engine: the k_random_go group and the k_replay group each get their own replicas
    rp = default_trace.replay(seed=44)
    keep = list(range(0, default_trace.num_nodes, 3))
    nodes = helpers.subset_nodes(rp, keep)
    n_ev = 2500
    states = [default_trace.go_state(seed=s) for s in (44, 45, 46)]
    got, _, _ = run_engine(default_trace, nodes, rp.events, n_ev, states, gpusel=gpusel, extra_hash=True)
    for r, st in enumerate(states):
        want, _, _ = oracle(default_trace, rp, keep, n_ev, st, gpusel=gpusel)
        assert got[r] == want, r
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    hashed, _, _ = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                helpers.oracle_events(default_trace, rp, n_ev), policy=O.POL_RANDOM,
                                gpu_sel=SEL[gpusel], seed=5, threads=8)
    assert got[3] == hashed and got[3] != got[0]


def test_deletes_report_and_final_state(default_trace):
    rp = default_trace.replay(seed=9)
    keep = list(range(1, default_trace.num_nodes, 4))
    nodes = helpers.subset_nodes(rp, keep)
    evs, oev = helpers.delete_stream(default_trace, rp, 1500, 0.3, seed=4)
    st = default_trace.go_state(seed=9)
    got, reps, final = run_engine(default_trace, nodes, evs, len(evs), [st], report=True)
    want, wstate, wrep = oracle(default_trace, rp, keep, len(evs), st, report=True, events=oev)
    assert got[0] == want
    assert any(r[4] == ksim.DELETED and r[0] >= 0 for r in got[0])
    for i, (g, w) in enumerate(zip(reps[0], wrep)):
        assert g["frag_bins"] == w["frag_bins_exact"], i
        for k in ("used_nodes", "used_gpus", "used_gpu_milli", "used_cpu_milli", "arrived_gpu_milli"):
            assert g[k] == w[k], (i, k)
    for (cu, mu, pu, gu), node, (cl, ml, pods, gl) in zip(final[0], nodes, wstate):
        assert node.cpu_alloc_milli - cu == cl and node.mem_alloc_mib - mu == ml and pu == pods


def test_nodes_beyond_lds(default_trace):
    # 6000 nodes (the synthetic generator): the records stay in HBM (k_random_go<false>)
    t = default_trace.synthetic(6000, 800, seed=3)
    rp = t.replay(seed=3, tune_ratio=0.0, shuffle=False)
    st = t.go_state(seed=3, tune_ratio=0.0, shuffle=False)
    n_ev = min(rp.n, 800)
    got, _, _ = run_engine(t, rp.nodes, rp.events, n_ev, [st])
    want, _, _ = oracle(t, rp, list(range(t.num_nodes)), n_ev, st)
    assert got[0] == want


def test_unsupported_paths_refuse(default_trace):
    rp = default_trace.replay(seed=42)
    st = default_trace.go_state(seed=42)
    arr, n = default_trace.typical()
    for kw, sel in (({"run_mode": 1}, "random"), ({}, "FGD")):
        eng = ksim.Engine(default_trace.num_nodes, 1, **kw)
        eng.set_nodes(0, rp.nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "Random", gpusel=sel)
        eng.set_go_stream(0, st)
        eng.load_events(0, rp.events, 100)
        with pytest.raises(ksim.KsimError) as ei:
            eng.run()
        assert ei.value.code == ksim.KSIM_ENOTSUP
        eng.set_go_stream(0, None)  # back to the hash contract: runs
        eng.run()
        eng.close()


def test_go_stream_sweep_near_expected():
    # the paper's Random experiments (openb default, 10 seeds) on the Go-stream draw structure: the
    # 10-seed mean curves near the reference's (its own Random runs are timing-dependent)
    sw = SW.Sweep(SW.plan(traces=["openb_pod_list_default"], policies=("01-Random",)), random_stream="go")
    sw.run()
    curves = sw.curves()
    sw.close()
    for kind, csv in (("alloc", ALLO), ("frag", FRAG)):
        ours = SW.mean_curve(curves, "openb_pod_list_default", "01-Random", kind)
        ref = SW.expected_mean_curve(csv, "openb_pod_list_default", "01-Random")
        keys = [k for k in ours if k in ref]
        assert len(keys) >= 125
        dev = max(abs(ours[k] - ref[k]) for k in keys)
        print("Go-stream Random vs expected_results (%s): worst 10-seed mean deviation %.3f" % (kind, dev))
        assert dev <= 1.5, (kind, dev)
