"""GPU parity of the memoised FGD replays -- k_memo (run_mode 3, keys in LDS over K workgroups) and
k_hmemo (run_mode 5, keys in HBM; one workgroup per replica, or with wgs_per_replica > 1 / clusters
over 4096 nodes the wide form: K workgroups each owning a slice of ranks, one exchange per pod) --
against the oracle and against the scanning replay (k_replay, run_mode 2).

k_memo keeps the key of every (pod class, node) pair and recomputes only the node the previous
event changed; in decider mode (run_mode 4) workgroup 0 decides every event from the class owners'
top lists, kLag events old, plus the fresh keys of the nodes changed since; the bar is the same as every other path: bit-exact (node, GPU set, score, feasible
count, status) per event and the same final cluster state.  Every test needs a gfx950 device.
"""
import numpy as np
import pytest

import helpers
import ksim
import pyoracle as O
from test_gpu_parity import assert_same, engine_run, oracle_run

pytestmark = pytest.mark.gpu

MEMO, SCAN, DECIDER, HMEMO = 3, 2, 4, 5
MODES = pytest.mark.parametrize("mode", [MEMO, DECIDER, HMEMO], ids=["memo", "decider", "hmemo"])


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


@MODES
def test_memo_full_openb_fgd(default_trace, mode):
    # C2 at one seed: 10 953 events on 1213 nodes, memo == oracle == k_replay
    rp = default_trace.replay(seed=42)
    res, state = engine_run(default_trace, rp, None, rp.n, "FGD", run_mode=mode)
    want, want_state, _ = oracle_run(default_trace, rp, None, rp.n, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, None)
    scan, _ = engine_run(default_trace, rp, None, rp.n, "FGD", run_mode=SCAN)
    assert res == scan


@MODES
@pytest.mark.parametrize("wgs", [3, 4, 8, 25, 64])
def test_memo_workgroups_invariance(default_trace, wgs, mode):
    # any number of class-owning workgroups per replica gives the same decisions
    rp = default_trace.replay(seed=6)
    keep = list(range(0, default_trace.num_nodes, 3))
    res, state = engine_run(default_trace, rp, keep, 1500, "FGD", run_mode=mode, wgs=wgs)
    want, want_state, _ = oracle_run(default_trace, rp, keep, 1500, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)


@MODES
@pytest.mark.parametrize("trace_name", ["gpuspec33", "multigpu50", "gpushare100", "cpu250"])
def test_memo_other_traces(trace_name, mode):
    # gpuspec33: 457 pod classes and typed typical pods (the NA bin)
    t = ksim.Trace.openb(trace_name)
    rp = t.replay(seed=43)
    keep = list(range(1, t.num_nodes, 3))
    n_ev = min(rp.n, 2500)
    res, state = engine_run(t, rp, keep, n_ev, "FGD", run_mode=mode)
    want, want_state, _ = oracle_run(t, rp, keep, n_ev, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)


@pytest.mark.parametrize("memo_mode", [MEMO, DECIDER, HMEMO], ids=["memo", "decider", "hmemo"])
def test_memo_ten_replicas_ragged(default_trace, memo_mode):
    # the C2 layout (10 seeds, one engine) with ragged stream lengths: memo == k_replay
    arr, n = default_trace.typical()
    outs = {}
    for mode in (memo_mode, SCAN):
        eng = ksim.Engine(default_trace.num_nodes, 10, run_mode=mode)
        for r in range(10):
            rp = default_trace.replay(seed=42 + r)
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, "FGD")
            eng.load_events(r, rp.events, rp.n - 97 * r)
        eng.run()
        outs[mode] = [eng.results(r) for r in range(10)]
        if mode == memo_mode == HMEMO:
            assert eng.last_run_wgs() == 1 and eng.last_run_path() == "k_hmemo"
        elif mode == memo_mode:
            assert eng.last_run_wgs() >= 8 and eng.last_run_path() == "k_memo"
        eng.close()
    for r in range(10):
        assert outs[memo_mode][r] == outs[SCAN][r], "replica %d" % r


def test_memo_mixed_policies(default_trace):
    # FGD replicas take k_memo, the others k_replay, in one run (run_mode 0 = auto)
    cfgs = [(42, "FGD", O.POL_FGD, O.SEL_FGD), (43, "BestFit", O.POL_BESTFIT, O.SEL_BEST),
            (45, "FGD", O.POL_FGD, O.SEL_FGD)]
    keep = list(range(0, default_trace.num_nodes, 4))
    arr, n = default_trace.typical()
    eng = ksim.Engine(len(keep), len(cfgs))
    rps = []
    for r, (seed, name, _, _) in enumerate(cfgs):
        rp = default_trace.replay(seed=seed)
        rps.append(rp)
        eng.set_nodes(r, helpers.subset_nodes(rp, keep))
        eng.set_typical(r, arr, n)
        eng.set_policy(r, name)
        eng.load_events(r, rp.events, 1100 + 100 * r)
    eng.run()
    for r, (seed, name, pol, sel) in enumerate(cfgs):
        want, _, _ = oracle_run(default_trace, rps[r], keep, 1100 + 100 * r, pol, sel)
        assert eng.results(r) == want, "replica %d (%s)" % (r, name)
    eng.close()


@MODES
def test_memo_deletions(default_trace, mode):
    rp = default_trace.replay(seed=9)
    keep = list(range(0, default_trace.num_nodes, 9))
    evs, oev = helpers.delete_stream(default_trace, rp, 900, 0.3, seed=0)
    arr, n = default_trace.typical()
    eng = ksim.Engine(len(keep), 1, run_mode=mode, wgs_per_replica=6)
    eng.set_nodes(0, helpers.subset_nodes(rp, keep))
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, evs, len(evs))
    eng.run()
    got = eng.results(0)
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    want, want_state, _ = O.run_events(onodes, helpers.oracle_typical(default_trace), oev, policy=O.POL_FGD,
                                       gpu_sel=O.SEL_FGD, threads=16)
    assert_same(got, want, eng.nodes(0), want_state, keep)
    assert any(r[4] == ksim.DELETED and r[0] >= 0 for r in got)
    eng.close()


@MODES
def test_memo_tiny_cluster(default_trace, mode):
    # 3 nodes, more workgroups than classes and nodes; the cluster fills up and pods fail
    rp = default_trace.replay(seed=3)
    keep = [5, 600, 1100]
    res, state = engine_run(default_trace, rp, keep, 400, "FGD", run_mode=mode, wgs=16)
    want, want_state, _ = oracle_run(default_trace, rp, keep, 400, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, keep)
    assert any(r[4] == ksim.UNSCHEDULABLE for r in res)


@MODES
def test_memo_rerun_same_results(default_trace, mode):
    # run() restarts from the set_nodes state: two runs of one engine agree
    rp = default_trace.replay(seed=44)
    arr, n = default_trace.typical()
    eng = ksim.Engine(default_trace.num_nodes, 1, run_mode=mode)
    eng.set_nodes(0, rp.nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, "FGD")
    eng.load_events(0, rp.events, 3000)
    eng.run()
    a = eng.results(0)
    eng.run()
    assert eng.results(0) == a
    eng.close()


def test_memo_not_applicable_is_loud(default_trace):
    # one workgroup cannot hold 151 classes x 404 nodes of keys: run_mode 3 refuses (no silent scan)
    rp = default_trace.replay(seed=6)
    keep = list(range(0, default_trace.num_nodes, 3))
    with pytest.raises(ksim.KsimError):
        engine_run(default_trace, rp, keep, rp.n, "FGD", run_mode=MEMO, wgs=1)


def test_hmemo_when_kmemo_does_not_fit(default_trace):
    # two workgroups per replica cannot hold 151 classes x 1213 nodes of keys in LDS, so k_memo does
    # not fit; auto mode takes k_hmemo (one workgroup per replica), bit-exact with k_replay
    arr, n = default_trace.typical()
    R = 30
    outs = {}
    for mode in (0, SCAN):
        eng = ksim.Engine(default_trace.num_nodes, R, run_mode=mode, wgs_per_replica=2 if mode == 0 else 0)
        for r in range(R):
            rp = default_trace.replay(seed=100 + r)
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, "FGD")
            eng.load_events(r, rp.events, 600 + 7 * r)
        eng.run()
        if mode == 0:
            assert eng.last_run_path() == "k_hmemo"
        outs[mode] = [eng.results(r) for r in range(R)]
        eng.close()
    assert outs[0] == outs[SCAN]


@pytest.mark.parametrize("wgs", [2, 7, 19, 64])
def test_hmemo_wide_vs_oracle(default_trace, wgs):
    # the wide k_hmemo: ceil(1213 / S) workgroups of S ranks (S a multiple of 64), one exchange per pod
    rp = default_trace.replay(seed=48)
    n_ev = 3000
    res, state = engine_run(default_trace, rp, None, n_ev, "FGD", run_mode=HMEMO, wgs=wgs)
    want, want_state, _ = oracle_run(default_trace, rp, None, n_ev, O.POL_FGD, O.SEL_FGD)
    assert_same(res, want, state, want_state, None)


def test_hmemo_wide_replicas_and_path(default_trace):
    # three replicas x K workgroups in one cooperative launch; the engine reports the path and K
    arr, n = default_trace.typical()
    outs = {}
    for mode, wgs in ((HMEMO, 5), (SCAN, 0)):
        eng = ksim.Engine(default_trace.num_nodes, 3, run_mode=mode, wgs_per_replica=wgs)
        for r in range(3):
            rp = default_trace.replay(seed=60 + r)
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, "FGD")
            eng.load_events(r, rp.events, 2000 + 300 * r)
        eng.run()
        if mode == HMEMO:
            assert eng.last_run_path() == "k_hmemo" and eng.last_run_wgs() == 5
        outs[mode] = [eng.results(r) for r in range(3)]
        eng.close()
    assert outs[HMEMO] == outs[SCAN]


@pytest.mark.parametrize("wgs", [0, 5])
def test_hmemo_cluster_report(default_trace, wgs):
    # the per-event report from k_hmemo's snapshots equals k_replay's (exact fixed-point sums)
    rp = default_trace.replay(seed=47)
    arr, n = default_trace.typical()
    reps = {}
    for mode in (HMEMO, SCAN):
        eng = ksim.Engine(default_trace.num_nodes, 1, run_mode=mode, wgs_per_replica=wgs if mode == HMEMO else 0)
        eng.set_nodes(0, rp.nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "FGD")
        eng.set_report(True)
        eng.load_events(0, rp.events, 4000)
        eng.run()
        reps[mode] = (eng.results(0), eng.reports(0))
        eng.close()
    assert reps[HMEMO] == reps[SCAN]


@pytest.mark.parametrize("form", ["lean", "report", "deletes"])
def test_memo_keys_in_hbm(form):
    # r06: gpuspec33 (457 classes, score groups of up to 60 classes) at 25 workgroups per replica: its keys do not
    # fit in LDS beside the cluster, so k_memo keeps them in HBM and splits the large groups over workgroups --
    # bit-exact against the oracle in the lean form, the lean form with the report's stores (against k_hmemo's
    # reports) and the general one (a create / delete stream)
    t = ksim.Trace.openb("gpuspec33")
    rp = t.replay(seed=43)
    arr, n = t.typical()
    if form == "deletes":
        evs, oev = helpers.delete_stream(t, rp, 1800, 0.3, seed=2)
        n_ev = len(evs)
        want, want_state, _ = O.run_events(helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), oev, policy=O.POL_FGD,
                                           gpu_sel=O.SEL_FGD, threads=16)
    else:
        evs, n_ev = rp.events, 2500
        want, want_state, _ = oracle_run(t, rp, None, n_ev, O.POL_FGD, O.SEL_FGD)
    outs = {}
    for mode, wgs in ((MEMO, 25), (HMEMO, 1)):
        eng = ksim.Engine(t.num_nodes, 1, run_mode=mode, wgs_per_replica=wgs)
        eng.set_nodes(0, rp.nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "FGD")
        if form == "report":
            eng.set_report(True)
        eng.load_events(0, evs, n_ev)
        eng.run()
        assert eng.last_run_kernels() == (["k_memo_hkeys"] if mode == MEMO else ["k_hmemo"])
        assert eng.last_run_wgs() == wgs
        outs[mode] = (eng.results(0), eng.nodes(0), eng.reports(0) if form == "report" else None)
        eng.close()
    assert_same(outs[MEMO][0], want, outs[MEMO][1], want_state, None)
    if form == "report":
        assert outs[MEMO][2] == outs[HMEMO][2]


def test_hmemo_per_model_tables_that_do_not_fit():
    # r05 advisor: a typed replica whose per-model tables exceed their 12-bit offsets (25 GPU models x 200 GPU typical
    # pods accepting every model = 5 000 entries) runs k_hmemo on the whole table, bit-exact, instead of refusing it
    from fuzz_cases import _mask, make_case
    from test_gpu_fuzz import check_state, run_engine
    models = [chr(ord("a") + i) for i in range(25)]  # one-letter names: the oracle keeps a spec in 64 bytes
    case = make_case(11, 400, 1500, models=models)
    vocab = models + ["H100"]
    assert len({n["model"] for n in case["onodes"] if n["gpu"]}) == 25
    spec = "|".join(models)
    rnd = np.random.default_rng(3)
    otyp = [(int(c), 0, 0, "", 0.002) for c in (500, 1000, 4000, 8000)]
    for k in range(200):
        milli, num = (int(rnd.choice([100, 250, 500, 700])), 1) if k % 2 else (1000, int(rnd.choice([1, 2, 4, 8])))
        otyp.append((int(rnd.choice([0, 4000, 16000])), milli, num, spec, 0.004))
    typ = (ksim.Typical * len(otyp))()
    for i, (cpu, milli, num, sp, freq) in enumerate(otyp):
        typ[i].cpu_milli, typ[i].gpu_milli, typ[i].gpu_count = cpu, milli, num
        typ[i].type_mask, typ[i].freq = _mask(sp, vocab), freq
    case.update(typical=typ, typical_n=len(otyp), otypical=otyp)
    want, want_state, _ = O.run_events(case["onodes"], otyp, case["oevents"], policy=O.POL_FGD, gpu_sel=O.SEL_FGD,
                                       threads=16)
    got, state = run_engine(case, "FGD", HMEMO, wgs=1)  # run_mode 5: k_hmemo or an error, never another path
    assert got == want
    check_state(state, want_state)


@pytest.mark.parametrize("knobs", [{"KSIM_VARIANT": "hprune=-1"}, {"KSIM_VARIANT": "hmodel=0"},
                                   {"KSIM_VARIANT": "hmodel=0,hprune=100000"}, {"KSIM_VARIANT": "hl2=1"}],
                         ids=["prune-all", "whole-table", "r04-form", "l2"])
@pytest.mark.parametrize("trace_name", ["gpuspec33", "gpuspec10", "default"])
def test_hmemo_list_and_table_forms(trace_name, knobs, monkeypatch):
    # r05: k_hmemo's F list without the groups no class of which passes Filter on d (by default for tables of
    # more than 64 typical pods; -1: every replica), and per GPU model the typical table cut to the pods that
    # accept the model plus the precomputed NA bin (typed replicas; hmodel=0 the whole table), and the
    # per-(class, block) second maxima (hl2=1: one workgroup per replica only, compiled out of the wide form):
    # every form decides as the oracle does, one workgroup per replica and the wide form
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    t = ksim.Trace.openb(trace_name)
    rp = t.replay(seed=44)
    n_ev = min(rp.n, 3000)
    want, want_state, _ = oracle_run(t, rp, None, n_ev, O.POL_FGD, O.SEL_FGD)
    for wgs in (0, 6):
        res, state = engine_run(t, rp, None, n_ev, "FGD", run_mode=HMEMO, wgs=wgs)
        assert_same(res, want, state, want_state, None)


@pytest.mark.parametrize("form", ["lean", "report", "deletes"])
def test_memo_replicas_at_their_own_widths(form):
    # r06: one k_memo launch holding replicas of different widths (ksim_engine_set_replica_wgs per replica; the
    # block map MemoArgs::wg_map): three seeds at 4, 12 and 25 workgroups, each bit-exact against the oracle in the
    # lean form, with the report's stores (against the one-workgroup k_hmemo's reports) and in the general form
    t = ksim.Trace.openb("default")
    arr, n = t.typical()
    widths = (4, 12, 25)
    cases = []
    for s in (42, 45, 49):
        rp = t.replay(seed=s)
        if form == "deletes":
            evs, oev = helpers.delete_stream(t, rp, 1500, 0.3, seed=s)
            n_ev = len(evs)
            want = O.run_events(helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), oev, policy=O.POL_FGD,
                                gpu_sel=O.SEL_FGD, threads=16)
        else:
            evs, n_ev = rp.events, 2000
            want = oracle_run(t, rp, None, n_ev, O.POL_FGD, O.SEL_FGD)
        cases.append((rp, evs, n_ev, want))
    outs = {}
    for mode in (MEMO, HMEMO):
        eng = ksim.Engine(t.num_nodes, len(cases), run_mode=mode, wgs_per_replica=0 if mode == MEMO else 1)
        for r, (rp, evs, n_ev, _) in enumerate(cases):
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, "FGD")
            if mode == MEMO:
                eng.set_replica_wgs(r, widths[r])
            eng.load_events(r, evs, n_ev)
        if form == "report":
            eng.set_report(True)
        eng.run()
        kern = eng.last_run_kernels()
        assert kern[0] in (("k_memo", "k_memo_hkeys") if mode == MEMO else ("k_hmemo",)), kern
        outs[mode] = [(eng.results(r), eng.nodes(r), eng.reports(r) if form == "report" else None)
                      for r in range(len(cases))]
        eng.close()
    for r, (_, _, _, (want, want_state, _)) in enumerate(cases):
        assert_same(outs[MEMO][r][0], want, outs[MEMO][r][1], want_state, None)
        if form == "report":
            assert outs[MEMO][r][2] == outs[HMEMO][r][2], r
