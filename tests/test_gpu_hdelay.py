"""Hand-over stress for the memoised FGD kernels (KSIM_TEST=hdelay=<mask>, round-3 verdict item 1).

k_memo hands its critical F over through an LDS counter (the owner's waves 1-9 to wave 0) and otherwise
joins on barriers; its delay points: 1 every wave before the end-of-step barrier (wave 0 before it receives
the granule), 2 the owner's critical waves before their F, 4 every wave at the step start.  The lean kernel
with them compiled in (a hdelay mask selects it) runs the dead-class skip too.

k_hmemo has no workgroup barrier inside a step: wave 0 (the event's own class, the decision, the Bind) and
waves 1-15 (every other class's refresh) hand work over through LDS counters and double-buffered state,
and join once, at the end-of-step barrier.  A wave that reads something late -- after another wave of the
same step already wrote the next step's value -- is the failure this design must exclude; r03 shipped one
(the dead-class set: a late bulk wave read the skip condition after wave 0 had marked the class dead,
skipped the step and stalled the bulk).  The delays make the late orders the common ones:
the general instantiation sleeps 0-3 x ~3.4 us at the hand-over points on about half the steps (a hash of
step, wave and workgroup; ksim_hmemo.hpp hdelay).  Every run here must finish without a bounded-wait
failure (run() raises KSIM_ESTATE on one) and give the decisions k_replay / the oracle give.
"""
import pytest

import helpers
import ksim
import pyoracle as O

pytestmark = pytest.mark.gpu

ALL = "0x1f"  # every delay point: bulk before the skip read, wave 1 before its list, wave 0 before its decision,
              # the class waves before the class pass, the F waves before item 0's F hand-over (the group keys)
SEEDS = list(range(42, 52))


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def c2_engine(trace, seeds, run_mode, wgs=0, n_ev=None):
    arr, n = trace.typical()
    eng = ksim.Engine(trace.num_nodes, len(seeds), run_mode=run_mode, wgs_per_replica=wgs)
    for r, s in enumerate(seeds):
        rp = trace.replay(seed=s, tune_ratio=1.3, shuffle=True)
        eng.set_nodes(r, rp.nodes)
        eng.set_typical(r, arr, n)
        eng.set_policy(r, "FGD")
        eng.load_events(r, rp.events, rp.n if n_ev is None else min(n_ev, rp.n))
    return eng


@pytest.fixture(scope="module")
def c2_replay(default_trace):
    """The C2 job's decisions on k_replay (run_mode 2: every node scanned per pod, no memo)."""
    eng = c2_engine(default_trace, SEEDS, 2)
    try:
        eng.run()
        return [eng.results(r) for r in range(len(SEEDS))]
    finally:
        eng.close()


@pytest.mark.parametrize("hpf", ["0", "1", "3"])
def test_hmemo_c2_delays(default_trace, c2_replay, monkeypatch, hpf):
    # the C2 job on k_hmemo at one workgroup per replica (run_mode 5), every delay point on, with wave 0
    # listing the next refresh (hpf=1) and also touching its flagged rows (=3) or not (0)
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % ALL)
    monkeypatch.setenv("KSIM_VARIANT", "hpf=%s" % hpf)
    eng = c2_engine(default_trace, SEEDS, 5)
    try:
        eng.run()
        assert eng.last_run_path() == "k_hmemo" and eng.last_run_wgs() == 1
        got = [eng.results(r) for r in range(len(SEEDS))]
    finally:
        eng.close()
    for r in range(len(SEEDS)):
        assert got[r] == c2_replay[r], "seed %d differs from k_replay" % SEEDS[r]


def test_hmemo_c2_seed_vs_oracle_with_delays(default_trace, monkeypatch):
    # one full seed against the oracle itself (k_replay is pinned the same way, tests/test_gpu_parity.py)
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % ALL)
    rp = default_trace.replay(seed=42, tune_ratio=1.3, shuffle=True)
    eng = c2_engine(default_trace, [42], 5)
    try:
        eng.run()
        got = eng.results(0)
    finally:
        eng.close()
    want, _, _ = O.run_events(helpers.oracle_nodes(default_trace, rp), helpers.oracle_typical(default_trace),
                              helpers.oracle_events(default_trace, rp), policy=O.POL_FGD, gpu_sel=O.SEL_FGD,
                              threads=16)
    assert got == want


@pytest.mark.parametrize("hpf", ["1", "5"])
def test_hmemo_wide_delays(default_trace, c2_replay, monkeypatch, hpf):
    # the wide form (K = 7 co-resident workgroups per replica, the granule exchange per pod) on four C2 seeds;
    # hpf=5: the workgroup that binds lists the next refresh on its wave 0 (bit 4: the wide form too)
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % ALL)
    monkeypatch.setenv("KSIM_VARIANT", "hpf=%s" % hpf)
    eng = c2_engine(default_trace, SEEDS[:4], 5, wgs=7)
    try:
        eng.run()
        assert eng.last_run_path() == "k_hmemo" and eng.last_run_wgs() == 7
        got = [eng.results(r) for r in range(4)]
    finally:
        eng.close()
    assert got == c2_replay[:4]


@pytest.fixture(scope="module")
def c5():
    base = ksim.Trace.openb("default")
    t = base.synthetic(100_000, 1_000_000, seed=0)
    rp = t.replay(seed=1, tune_ratio=0.0, shuffle=False)
    return t, rp


def _c5_run(t, rp, n_ev, run_mode):
    arr, n = t.typical()
    eng = ksim.Engine(t.num_nodes, 1, run_mode=run_mode)
    try:
        eng.set_nodes(0, rp.nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "FGD")
        eng.load_events(0, rp.events, n_ev)
        eng.run()
        return eng.results(0), eng.last_run_path(), eng.last_run_wgs()
    finally:
        eng.close()


def test_hmemo_c5_prefix_delays(c5, monkeypatch):
    # C5's wide k_hmemo (63 workgroups of 1600 ranks) on a 4 000-event prefix, every delay point on
    t, rp = c5
    n_ev = 4000
    want, _, _ = _c5_run(t, rp, n_ev, 2)
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % ALL)
    got, path, k = _c5_run(t, rp, n_ev, 0)
    assert path == "k_hmemo" and k == 63
    assert got == want


def test_hmemo_shard_group_delays(c5, monkeypatch):
    # the in-process node-sharded group (3 shards' slices in one launch, one exchange per pod)
    import ksim.shard as SH
    t, rp = c5
    n_ev = 3000
    want, _, _ = _c5_run(t, rp, n_ev, 2)
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % ALL)
    g = SH.ShardGroup(rp.nodes, t.typical(), 3)
    try:
        g.load_events(rp.events, n_ev)
        g.run()
        assert g.engines[0].last_run_wgs() >= 1  # the k_hmemo slices, not the k_step path
        assert g.results() == want
    finally:
        g.close()


@pytest.mark.parametrize("mask", ["0x7", "0x1", "0x6"])
def test_memo_c2_delays(default_trace, c2_replay, monkeypatch, mask):
    # the C2 job on k_memo (run_mode 3: 25 co-resident workgroups per replica), the lean kernel with the delays
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % mask)
    eng = c2_engine(default_trace, SEEDS, 3)
    try:
        eng.run()
        assert eng.last_run_path() == "k_memo" and eng.last_run_wgs() == 25
        got = [eng.results(r) for r in range(len(SEEDS))]
    finally:
        eng.close()
    for r in range(len(SEEDS)):
        assert got[r] == c2_replay[r], "seed %d differs from k_replay" % SEEDS[r]


def test_memo_deletes_report_delays(default_trace, monkeypatch):
    # the general k_memo (a create / delete stream with the per-event report) with every delay point on
    monkeypatch.setenv("KSIM_TEST", "hdelay=%s" % "0x7")
    rp = default_trace.replay(seed=44, tune_ratio=1.3, shuffle=True)
    keep = list(range(0, default_trace.num_nodes, 3))
    evs, oev = helpers.delete_stream(default_trace, rp, 1500, p_delete=0.3, seed=5)
    arr, n = default_trace.typical()
    eng = ksim.Engine(len(keep), 1, run_mode=3)
    try:
        eng.set_report(True)
        eng.set_nodes(0, helpers.subset_nodes(rp, keep))
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "FGD")
        eng.load_events(0, evs, len(evs))
        eng.run()
        assert eng.last_run_path() == "k_memo"
        got = eng.results(0)
    finally:
        eng.close()
    want, _, _ = O.run_events(helpers.oracle_subset(default_trace, rp, keep), helpers.oracle_typical(default_trace),
                              oev, policy=O.POL_FGD, gpu_sel=O.SEL_FGD, threads=16)
    assert got == want
