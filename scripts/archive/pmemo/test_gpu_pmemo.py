"""GPU parity of k_pmemo (run_mode 6): the pipelined memoised FGD replay on node slices of <= 64 ranks
(ksim_pmemo.hpp).  Each workgroup keeps the key of every (score group, slot) pair of its slice, evaluates
the next pod step while the previous step's exchange is in flight (its candidate as it is and in the
virtual slot with the pending Bind applied), and refreshes a committed node's stale keys in the
background.  Bar: bit-exact against the oracle (node, GPU set, score, feasible count, status per event,
final cluster state) and equal to the scanning replay (k_replay).  Every test needs a gfx950 device.
"""
import pytest

import helpers
import ksim
import pyoracle as O
from test_gpu_parity import assert_same, engine_run, oracle_run

pytestmark = pytest.mark.gpu

PMEMO, SCAN = 6, 2


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def _state(nodes):
    return [(s.cpu_used_milli, s.mem_used_mib, s.pods_used, tuple(s.gpu_used_milli)) for s in nodes]


def test_pmemo_full_openb_fgd(default_trace):
    # C2 at one seed: 10 953 events on 1213 nodes over 64 workgroups of <= 19 slots
    rp = default_trace.replay(seed=42)
    res, state = engine_run(default_trace, rp, None, rp.n, "FGD", run_mode=PMEMO)
    want, want_state, _ = oracle_run(default_trace, rp, None, rp.n, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, None)


@pytest.mark.parametrize("wgs", [7, 8, 25, 64])
def test_pmemo_workgroups_invariance(default_trace, wgs):
    # any slicing (405 nodes: 58 .. 7 slots per workgroup) gives the oracle's decisions
    rp = default_trace.replay(seed=6)
    keep = list(range(0, default_trace.num_nodes, 3))
    res, state = engine_run(default_trace, rp, keep, 1500, "FGD", run_mode=PMEMO, wgs=wgs)
    want, want_state, _ = oracle_run(default_trace, rp, keep, 1500, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)


def test_pmemo_single_workgroup(default_trace):
    # K = 1 (no exchange): a 60-node cluster in one workgroup, filled past saturation
    rp = default_trace.replay(seed=9)
    keep = list(range(5, default_trace.num_nodes, 20))[:60]
    res, state = engine_run(default_trace, rp, keep, 900, "FGD", run_mode=PMEMO, wgs=1)
    want, want_state, _ = oracle_run(default_trace, rp, keep, 900, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)
    assert any(r[4] == 1 for r in res)


@pytest.mark.parametrize("trace_name", ["gpuspec33", "multigpu50", "gpushare100", "cpu250"])
def test_pmemo_other_traces(trace_name):
    t = ksim.Trace.openb(trace_name)
    rp = t.replay(seed=43)
    keep = list(range(1, t.num_nodes, 3))
    n_ev = min(rp.n, 2500)
    res, state = engine_run(t, rp, keep, n_ev, "FGD", run_mode=PMEMO)
    want, want_state, _ = oracle_run(t, rp, keep, n_ev, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)


@pytest.mark.parametrize("sel", ["best", "worst", "random"])
def test_pmemo_gpu_selectors(default_trace, sel):
    rp = default_trace.replay(seed=12)
    keep = list(range(2, default_trace.num_nodes, 4))
    nodes = helpers.subset_nodes(rp, keep)
    arr, n = default_trace.typical()
    osel = {"best": O.SEL_BEST, "worst": O.SEL_WORST, "random": O.SEL_RANDOM}[sel]
    eng = ksim.Engine(len(keep), 1, run_mode=PMEMO)
    eng.set_nodes(0, nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD", gpusel=sel, seed=3)
    eng.load_events(0, rp.events, 2000)
    eng.run()
    res, state = eng.results(0), eng.nodes(0)
    assert eng.last_run_path() == "k_pmemo"
    eng.close()
    want, want_state, _ = oracle_run(default_trace, rp, keep, 2000, O.POL_FGD, osel, seed=3)
    assert_same(res, want, state, want_state, keep)


def test_pmemo_ten_replicas_ragged(default_trace):
    # the C2 layout (10 seeds, one engine, K = 25) with ragged stream lengths: k_pmemo == k_replay
    arr, n = default_trace.typical()
    outs = {}
    for mode in (PMEMO, SCAN):
        eng = ksim.Engine(default_trace.num_nodes, 10, run_mode=mode)
        for r in range(10):
            rp = default_trace.replay(seed=42 + r)
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, "FGD")
            eng.load_events(r, rp.events, rp.n - 97 * r)
        eng.run()
        outs[mode] = ([eng.results(r) for r in range(10)], [eng.nodes(r) for r in range(10)])
        if mode == PMEMO:
            assert eng.last_run_path() == "k_pmemo" and eng.last_run_wgs() == 25
        eng.close()
    for r in range(10):
        assert outs[PMEMO][0][r] == outs[SCAN][0][r], "replica %d" % r
        assert _state(outs[PMEMO][1][r]) == _state(outs[SCAN][1][r]), "replica %d" % r


def test_pmemo_refusals(default_trace):
    # deletes / the report / a cluster wider than 64 slots per workgroup: run_mode 6 refuses
    rp = default_trace.replay(seed=1)
    arr, n = default_trace.typical()
    eng = ksim.Engine(default_trace.num_nodes, 1, run_mode=PMEMO, wgs_per_replica=4)
    eng.set_nodes(0, rp.nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, rp.events, 100)
    with pytest.raises(ksim.KsimError):
        eng.run()
    eng.close()
