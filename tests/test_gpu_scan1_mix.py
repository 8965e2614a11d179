"""The cheap policies' single-workgroup groups as ONE k_scan1_mix launch.

A concurrent run (the paper sweep's shape: every group at one workgroup per replica) gives the
BestFit, DotProduct (merge / max), GpuPacking, GpuClustering and hash-Random replicas one launch with
the policy chosen per workgroup, longest stream first, on one side stream.  Bar: every event and the
final state bit-exact against the oracle (the same device functions as k_scan1 / k_replay), with and
without the merge (KSIM_VARIANT=scan1_mix=0: one k_scan1 launch per policy).
"""
import pytest

import helpers
import ksim
import pyoracle as O

pytestmark = pytest.mark.gpu

SEED = 2
# (policy, oracle policy, oracle selector, events replayed: ragged so the longest-first order matters)
CASES = [("BestFit", O.POL_BESTFIT, O.SEL_BEST, None), ("DotProd", O.POL_DOTPROD, O.SEL_BEST, 3000),
         ("GpuPacking", O.POL_PACKING, O.SEL_BEST, None), ("GpuClustering", O.POL_CLUSTERING, O.SEL_BEST, 5000),
         ("Random", O.POL_RANDOM, O.SEL_RANDOM, None), ("BestFit", O.POL_BESTFIT, O.SEL_BEST, 700),
         ("GpuClustering", O.POL_CLUSTERING, O.SEL_BEST, None)]


@pytest.fixture(scope="module")
def trace():
    return ksim.Trace.openb("default")


def oracle(trace, rp, n_ev, pol, sel):
    return O.run_events(helpers.oracle_nodes(trace, rp), helpers.oracle_typical(trace),
                        helpers.oracle_events(trace, rp, n_ev), policy=pol, gpu_sel=sel, seed=SEED, threads=16)


def check_state(state, want_state):
    for i, (cpu_left, mem_left, pods, gl) in enumerate(want_state):
        s = state[i]
        assert s.cpu_alloc_milli - s.cpu_used_milli == cpu_left
        assert s.mem_alloc_mib - s.mem_used_mib == mem_left
        assert s.pods_used == pods
        assert [1000 - s.gpu_used_milli[g] if g < s.gpu_count else 0 for g in range(8)] == gl


@pytest.mark.parametrize("report", [False, True], ids=["plain", "report"])
@pytest.mark.parametrize("mix", ["1", "0"], ids=["mix", "per-policy"])
def test_cheap_groups_in_one_launch(trace, mix, report, monkeypatch):
    monkeypatch.setenv("KSIM_VARIANT", "scan1_mix=%s" % mix)
    rp = trace.replay(seed=44)
    arr, n = trace.typical()
    eng = ksim.Engine(trace.num_nodes, len(CASES), wgs_per_replica=1)
    try:
        if report:
            eng.set_report(True)
        for r, (name, _, _, n_ev) in enumerate(CASES):
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, name, seed=SEED)
            eng.load_events(r, rp.events, n_ev or rp.n)
        eng.run()
        launches, streams = eng.last_run_launches()
        assert eng.last_run_path() == "k_scan1"
        # merged: one launch on one side stream; else one k_scan1 per policy on the side streams
        assert (launches, streams) == ((1, 1) if mix == "1" else (5, min(4, 5)))
        if report:
            assert eng.last_report_ms() > 0  # the groups' report kernels ran (timed on their streams)
        got = [(eng.results(r), eng.nodes(r)) for r in range(len(CASES))]
        reps = [eng.report_arrays(r) for r in range(len(CASES))] if report else None
    finally:
        eng.close()
    for r, (name, pol, sel, n_ev) in enumerate(CASES):
        want, want_state, want_rep = oracle(trace, rp, n_ev or rp.n, pol, sel)
        res, state = got[r]
        bad = [i for i, (a, b) in enumerate(zip(res, want)) if a != b]
        assert len(res) == len(want) and not bad, (name, bad[:1])
        check_state(state, want_state)
    if report:
        # the sums of the per-event reports are exact (fix80): the two replays of one stream agree
        a, b = reps[0], reps[5]
        for k in a:
            assert (a[k][:700] == b[k][:700]).all(), k


def test_dotprod_other_configs_keep_their_own_launch(trace, monkeypatch):
    # a DotProduct replica outside the paper's merge / max configuration is not merged (the mix kernel
    # carries only the closed form): its group keeps a k_scan1 launch of its own, beside the merged one
    monkeypatch.setenv("KSIM_VARIANT", "scan1_mix=1")
    rp = trace.replay(seed=45)
    arr, n = trace.typical()
    names = ["BestFit", "DotProd", "GpuPacking"]
    eng = ksim.Engine(trace.num_nodes, 3, wgs_per_replica=1)
    try:
        for r, name in enumerate(names):
            eng.set_nodes(r, rp.nodes)
            eng.set_typical(r, arr, n)
            eng.set_policy(r, name, seed=SEED, **({"dim_ext": "share", "gpusel": "best"} if name == "DotProd" else {}))
            eng.load_events(r, rp.events, 2500)
        eng.run()
        assert eng.last_run_launches() == (2, 2)
        got = [eng.results(r) for r in range(3)]
    finally:
        eng.close()
    want = [oracle(trace, rp, 2500, O.POL_BESTFIT, O.SEL_BEST)[0],
            O.run_events(helpers.oracle_nodes(trace, rp), helpers.oracle_typical(trace),
                         helpers.oracle_events(trace, rp, 2500), policy=O.POL_DOTPROD, gpu_sel=O.SEL_BEST, seed=SEED,
                         threads=16, dim_ext=O.DIM_SHARE, norm=O.NORM_MAX)[0],
            oracle(trace, rp, 2500, O.POL_PACKING, O.SEL_BEST)[0]]
    assert got == want


def test_clustering_resumes_from_a_state_with_tags(trace, monkeypatch):
    # GpuClustering's presence bits are built from the tag counts set_nodes gives: replaying the second
    # half of a stream from the state the first half left (tag counts included) decides as the whole
    # replay does.  Both halves run in a mixed launch beside a BestFit replica.
    monkeypatch.setenv("KSIM_VARIANT", "scan1_mix=1")
    rp = trace.replay(seed=46)
    arr, n = trace.typical()
    k = 4000

    def run(nodes, events, count):
        eng = ksim.Engine(trace.num_nodes, 2, wgs_per_replica=1)
        try:
            for r, name in enumerate(["GpuClustering", "BestFit"]):
                eng.set_nodes(r, nodes)
                eng.set_typical(r, arr, n)
                eng.set_policy(r, name, seed=SEED)
                eng.load_events(r, events, count)
            eng.run()
            assert eng.last_run_launches() == (1, 1)
            return eng.results(0), eng.nodes(0)
        finally:
            eng.close()
    full, _ = run(rp.nodes, rp.events, rp.n)
    head, mid = run(rp.nodes, rp.events, k)
    assert any(sum(s.tag_count) > 0 for s in mid)
    tail_events = (ksim.Pod * (rp.n - k))()
    for i in range(rp.n - k):
        tail_events[i] = rp.events[k + i]
    tail, _ = run(mid, tail_events, rp.n - k)
    assert head == full[:k]
    assert [r[1:] for r in tail] == [r[1:] for r in full[k:]] and [r[0] for r in tail] == [r[0] for r in full[k:]]


@pytest.mark.parametrize("path", ["mix", "scan1", "replay", "replay-k4", "step"])
def test_nodes_beyond_max_spec_cpu(trace, path, monkeypatch):
    # nodes with more CPU than MaxSpecCpu (128 cores): BestFit's raw scores go below 0 (only -1 is a Score error,
    # best_fit_score.go:48-51; NormalizeScore spans any range) and DotProduct's can too (no NormalizeScore: the
    # framework's [0, 100] range check fails the cycle).  Every path -- k_scan1_mix, k_scan1 per policy, k_replay at one and four workgroups per replica (the
    # slices' exchange), k_step -- equals the oracle event by event.
    monkeypatch.setenv("KSIM_VARIANT", "scan1_mix=%d,scan1=%d" % (path == "mix", 0 if path.startswith("replay") else 2))
    rp = trace.replay(seed=47)
    arr, n = trace.typical()
    n_ev = 1500
    big = {i: (400000 if i % 6 == 0 else 150000) for i in range(0, trace.num_nodes, 3)}
    nodes = helpers.subset_nodes(rp, list(range(trace.num_nodes)))
    onodes = helpers.oracle_nodes(trace, rp)
    for i, c in big.items():
        nodes[i].cpu_alloc_milli = c
        onodes[i] = dict(onodes[i], cpu=c)
    names = [("BestFit", O.POL_BESTFIT), ("DotProd", O.POL_DOTPROD), ("GpuPacking", O.POL_PACKING)]
    got = []
    if path == "step":  # plugin-level calls: one replica per engine
        for name, _ in names:
            eng = ksim.Engine(trace.num_nodes, 1, run_mode=1)
            try:
                eng.set_nodes(0, nodes)
                eng.set_typical(0, arr, n)
                eng.set_policy(0, name, seed=SEED)
                eng.load_events(0, rp.events, n_ev)
                eng.run()
                got.append(eng.results(0))
            finally:
                eng.close()
    else:
        eng = ksim.Engine(trace.num_nodes, len(names), wgs_per_replica=4 if path == "replay-k4" else 1)
        try:
            for r, (name, _) in enumerate(names):
                eng.set_nodes(r, nodes)
                eng.set_typical(r, arr, n)
                eng.set_policy(r, name, seed=SEED)
                eng.load_events(r, rp.events, n_ev)
            eng.run()
            if path == "mix":
                assert eng.last_run_launches() == (1, 1)
            got = [eng.results(r) for r in range(len(names))]
        finally:
            eng.close()
    for r, (name, pol) in enumerate(names):
        want, _, _ = O.run_events(onodes, helpers.oracle_typical(trace), helpers.oracle_events(trace, rp, n_ev),
                                  policy=pol, gpu_sel=O.SEL_BEST, seed=SEED, threads=16)
        bad = [i for i, (a, b) in enumerate(zip(got[r], want)) if a != b]
        assert len(got[r]) == len(want) and not bad, (name, bad[:1], got[r][bad[0]] if bad else None,
                                                      want[bad[0]] if bad else None)
