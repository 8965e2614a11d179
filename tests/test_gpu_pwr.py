"""GPU parity of PWRScore and the weighted PWRScore + FGDScore combinations
(pkg/simulator/plugin/pwr_score.go; generate_run_scripts.py:31-42 "PWR", "PWR 500 FGD 500", ...).

The engine replays PWR replicas with the persistent k_replay (PWR: one key round per pod, the raw
score decides; PWR + FGD: one round carrying the cluster's min / max raw PWR score and each slice's
normalized weighted keys under two guessed ranges, a miss round when neither is the step's) and, with run_mode 1, on the per-pod path: k_step (Filter, raw PWR score, FGD
candidates) then k_step_pwr (NormalizeScore, weighted sum, selectHost, Reserve, Bind) in a hipGraph.
Bar: bit-exact against the oracle, event by event, and the same final cluster state, on every path.
Every test needs a gfx950 device.
"""
import pytest

import helpers
import ksim
import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


PATHS = {"k_replay": dict(), "k_replay-K1": dict(wgs_per_replica=1), "k_replay-K4": dict(wgs_per_replica=4),
         "k_step": dict(run_mode=1)}


def engine_run(trace, replay, keep, n_ev, policy, nodes=None, **kw):
    nodes = helpers.subset_nodes(replay, keep) if keep is not None else replay.nodes
    nn = len(keep) if keep is not None else trace.num_nodes
    arr, n = trace.typical()
    eng = ksim.Engine(nn, 1, **kw)
    eng.set_nodes(0, nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, policy)
    eng.set_power_model(0, trace.power_model())
    eng.load_events(0, replay.events, n_ev)
    eng.run()
    path = eng.last_run_path()
    res, state = eng.results(0), eng.nodes(0)
    eng.close()
    return res, state, path


def oracle_run(trace, replay, keep, n_ev, policy, threads=16):
    name, w = ksim.parse_policy(policy)
    pol = O.POL_PWR if name == "PWR" else O.POL_PWR_FGD
    sel = O.SEL_PWR if name == "PWR" else O.SEL_FGD
    onodes = helpers.oracle_nodes(trace, replay)
    if keep is not None:
        onodes = [onodes[i] for i in keep]
    w_pwr, w_fgd = w if w else (0, 0)
    return O.run_events(onodes, helpers.oracle_typical(trace), helpers.oracle_events(trace, replay, n_ev),
                        policy=pol, gpu_sel=sel, threads=threads, w_pwr=w_pwr, w_fgd=w_fgd)


def assert_same(res, want, state, want_state):
    bad = [i for i, (a, b) in enumerate(zip(res, want)) if a != b]
    assert len(res) == len(want) and not bad, "first mismatch at event %d: gpu %s oracle %s" % (
        bad[0], res[bad[0]], want[bad[0]])
    for i, (cpu_left, mem_left, pods, gl) in enumerate(want_state):
        s = state[i]
        assert s.cpu_alloc_milli - s.cpu_used_milli == cpu_left and s.pods_used == pods
        assert [1000 - s.gpu_used_milli[g] if g < s.gpu_count else 0 for g in range(8)] == gl


@pytest.mark.parametrize("run", sorted(PATHS))
@pytest.mark.parametrize("policy", ["PWR", "PWR 500 FGD 500", "PWR 100 FGD 900", "PWR 50 FGD 950"])
def test_subset_replay(default_trace, policy, run):
    rp = default_trace.replay(seed=42)
    keep = list(range(3, default_trace.num_nodes, 7))  # 173 nodes, every GPU model
    n_ev = 1500
    res, state, path = engine_run(default_trace, rp, keep, n_ev, policy, **PATHS[run])
    want, want_state, _ = oracle_run(default_trace, rp, keep, n_ev, policy)
    assert path == run.split("-")[0]
    assert_same(res, want, state, want_state)
    assert sum(1 for r in res if r[0] >= 0) > 300 and any(r[4] == 1 for r in res)  # fills up, then fails


@pytest.mark.parametrize("policy", ["PWR", "PWR 500 FGD 500"])
def test_full_trace(default_trace, policy):
    rp = default_trace.replay(seed=43)
    res, state, path = engine_run(default_trace, rp, None, rp.n, policy)
    assert path == "k_replay"
    want, want_state, _ = oracle_run(default_trace, rp, None, rp.n, policy)
    assert_same(res, want, state, want_state)


@pytest.mark.parametrize("run", ["k_replay", "k_replay-K1", "k_step"])
@pytest.mark.parametrize("policy", ["PWR", "PWR 500 FGD 500"])
def test_deletes_and_report(default_trace, policy, run):
    # a create / delete stream with the per-event cluster report on (k_replay's general instantiation)
    rp = default_trace.replay(seed=44)
    keep = list(range(1, default_trace.num_nodes, 5))
    evs, oev = helpers.delete_stream(default_trace, rp, 1000, p_delete=0.3, seed=3)
    arr, n = default_trace.typical()
    eng = ksim.Engine(len(keep), 1, **PATHS[run])
    try:
        eng.set_nodes(0, helpers.subset_nodes(rp, keep))
        eng.set_typical(0, arr, n)
        eng.set_policy(0, policy)
        eng.set_power_model(0, default_trace.power_model())
        eng.set_report(True)
        eng.load_events(0, evs, len(evs))
        eng.run()
        assert eng.last_run_path() == run.split("-")[0]
        got, state = eng.results(0), eng.nodes(0)
    finally:
        eng.close()
    name, w = ksim.parse_policy(policy)
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    w_pwr, w_fgd = w if w else (0, 0)
    want, want_state, _ = O.run_events(onodes, helpers.oracle_typical(default_trace), oev,
                                       policy=O.POL_PWR if name == "PWR" else O.POL_PWR_FGD,
                                       gpu_sel=O.SEL_PWR if name == "PWR" else O.SEL_FGD, threads=16,
                                       w_pwr=w_pwr, w_fgd=w_fgd)
    assert any(r[4] == 3 for r in got)
    assert_same(got, want, state, want_state)


def test_plugin_level_score_and_reserve(default_trace):
    # Score before NormalizeScore and the PWR GPU choice per node (the batch a Go PreScore shim
    # would store), then Reserve with gpuSelMethod "PWRScore"
    rp = default_trace.replay(seed=44)
    keep = list(range(0, default_trace.num_nodes, 11))
    eng = ksim.Engine(len(keep), 1)
    eng.set_nodes(0, helpers.subset_nodes(rp, keep))
    eng.set_policy(0, "PWR")
    eng.set_power_model(0, default_trace.power_model())
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    evs = helpers.oracle_events(default_trace, rp, 200)
    for k in range(0, 200, 17):
        feas, score, gpu = eng.filter_score(0, rp.events[k], step=k)
        e = evs[k]
        pr = O.pod_res(e["cpu"], e["milli"], e["num"], e["type"])
        for j, d in enumerate(onodes):
            if not feas[j]:
                continue
            nr = O.node_res(d["cpu"], [1000] * d["gpu"], d["gpu"], d["model"], d["cpu"])
            s, m, err = O.pwr_score(nr, pr)
            assert err == 0 and score[j] == s
            if e["num"] == 1 and e["milli"] < 1000:
                assert gpu[j] == m
    # Reserve on node 0 picks the PWR GPU; Unreserve restores the node
    share = next(k for k, e in enumerate(evs) if e["num"] == 1 and 0 < e["milli"] < 1000)
    mask = eng.reserve(0, rp.events[share], 0, step=share)
    assert mask == 1  # fresh node: every GPU costs the same, the first is kept
    eng.unreserve(0, rp.events[share], 0, mask)
    assert all(g == 0 for g in eng.nodes(0)[0].gpu_used_milli)
    eng.close()


def test_errors(default_trace):
    rp = default_trace.replay(seed=42)
    eng = ksim.Engine(default_trace.num_nodes, 1)
    eng.set_nodes(0, rp.nodes)
    eng.set_policy(0, "PWR")
    eng.load_events(0, rp.events, 10)
    with pytest.raises(ksim.KsimError) as ei:
        eng.run()  # no power model yet
    assert ei.value.code == ksim.KSIM_ESTATE
    with pytest.raises(ksim.KsimError):
        eng.set_policy(0, "FGD", gpusel="PWR")  # allocateGpuIdFunc has no PWRScore without the plugin
    eng.set_policy(0, "PWR 500 FGD 500")
    with pytest.raises(ksim.KsimError):
        eng.filter_score(0, rp.events[0])  # two plugins: no single plugin-level Score
    eng.close()


@pytest.mark.parametrize("env", [{"KSIM_VARIANT": "pf_memo=0"}, {"KSIM_TEST": "pf_memo_ver0=%d" % (0x3fff - 3)},
                                 {"KSIM_TEST": "pf_guess=0"}],
                         ids=["memo-off", "version-wrap", "no-guess"])
def test_pf_memo_off_and_version_wrap(default_trace, monkeypatch, env):
    # k_replay<PWR+FGD> keeps every class's Filter + Score of every slot in LDS while the slot's record is
    # unchanged (the default): without the memo, and with the slot versions starting three changes before
    # their 14-bit field wraps (every entry of a wrapping slot is forgotten first), the decisions stay the
    # oracle's -- the subset replay at the default K and at K = 1.  KSIM_TEST=pf_guess=0: no class ever has a
    # guessed NormalizeScore range, so every step with two or more feasible nodes takes the miss round (and its
    # owner the re-evaluation when its winner is not the virtual node)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rp = default_trace.replay(seed=45)
    keep = list(range(2, default_trace.num_nodes, 7))
    for kw in (dict(), dict(wgs_per_replica=1)):
        res, state, path = engine_run(default_trace, rp, keep, 1500, "PWR 500 FGD 500", **kw)
        want, want_state, _ = oracle_run(default_trace, rp, keep, 1500, "PWR 500 FGD 500")
        assert path == "k_replay"
        assert_same(res, want, state, want_state)
