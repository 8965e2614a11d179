"""Parity fuzz on adversarial synthetic clusters (tests/fuzz_cases.py): every policy through every
execution path -- auto (k_memo for FGD, k_replay for the rest), k_replay forced, k_step per pod
(hipGraph), k_hmemo forced for FGD (run_mode 5), k_memo forced for FGD -- bit-exact against the oracle per event (node, GPU set, score,
feasible count, status) and in the final cluster state.  Every test needs a gfx950 device.
"""
import pytest

import ksim
import pyoracle as O
from fuzz_cases import make_case
from test_gpu_parity import POLICIES

pytestmark = pytest.mark.gpu

# (seed, nodes, creations, delete probability)
CASES = [(1, 40, 500, 0.0), (2, 97, 900, 0.25), (3, 250, 1200, 0.1), (4, 7, 300, 0.4), (5, 1, 60, 0.3),
         (6, 600, 2000, 0.0)]
PATHS = [(0, "auto"), (2, "replay"), (1, "step"), (5, "hmemo"), (2, "replay-K1")]  # K1: k_scan1 when lean


def run_engine(case, policy, run_mode, seed=5, wgs=0):
    nn = len(case["onodes"])
    eng = ksim.Engine(nn, 1, run_mode=run_mode, wgs_per_replica=wgs)
    try:
        eng.set_nodes(0, case["nodes"])
        eng.set_typical(0, case["typical"], case["typical_n"])
        eng.set_policy(0, policy, seed=seed)
        eng.load_events(0, case["events"], case["n_events"])
        eng.run()
        return eng.results(0), eng.nodes(0)
    finally:
        eng.close()


def check_state(state, want_state):
    for i, (cpu_left, mem_left, pods, gl) in enumerate(want_state):
        s = state[i]
        assert (s.cpu_alloc_milli - s.cpu_used_milli, s.mem_alloc_mib - s.mem_used_mib, s.pods_used) == \
            (cpu_left, mem_left, pods), "node %d" % i
        assert [1000 - s.gpu_used_milli[g] if g < s.gpu_count else 0 for g in range(8)] == gl, "node %d" % i


@pytest.fixture(scope="module", params=CASES, ids=["s%d-n%d-e%d-d%g" % c for c in CASES])
def case(request):
    seed, n, e, pdel = request.param
    return make_case(seed, n, e, pdel)


@pytest.mark.parametrize("name,pol,sel", POLICIES, ids=[p[0] for p in POLICIES])
def test_fuzz_all_paths_vs_oracle(case, name, pol, sel):
    want, want_state, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=pol, gpu_sel=sel,
                                       seed=5, threads=16)
    for mode, label in PATHS:
        got, state = run_engine(case, name, mode, wgs=1 if label == "replay-K1" else 0)
        bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
        assert len(got) == len(want) and not bad, \
            "%s/%s: first mismatch at event %d: gpu %s oracle %s" % (name, label, bad[0], got[bad[0]], want[bad[0]])
        check_state(state, want_state)


def test_fuzz_memo_forced_fgd(case):
    # k_memo (run_mode 3) where its classes fit in LDS; it refuses loudly otherwise
    want, want_state, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=O.POL_FGD,
                                       gpu_sel=O.SEL_FGD, threads=16)
    try:
        got, state = run_engine(case, "FGD", 3)
    except ksim.KsimError as e:
        if e.code != ksim.KSIM_ENOTSUP:
            raise
        pytest.skip("k_memo does not fit this case")
    assert got == want
    check_state(state, want_state)


def test_fuzz_empty_event_stream():
    case = make_case(7, 30, 0)
    for mode, _ in PATHS:
        got, state = run_engine(case, "FGD", mode)
        assert got == []
        assert all(state[i].cpu_used_milli == 0 and state[i].pods_used == 0 for i in range(30))


def test_typical_table_over_engine_limit_is_loud():
    # the target-workload table lives in LDS, at most 256 entries (the reference traces: <= 127)
    tp = (ksim.Typical * 257)()
    for i in range(257):
        tp[i].cpu_milli, tp[i].gpu_milli, tp[i].gpu_count = 1000 + i, 100, 1
        tp[i].type_mask, tp[i].freq = ksim.KSIM_TYPE_ANY, 1.0 / 257
    eng = ksim.Engine(4, 1)
    try:
        with pytest.raises(ksim.KsimError):
            eng.set_typical(0, tp, 257)
        eng.set_typical(0, tp, 256)
    finally:
        eng.close()


REPORT_KEYS = ["used_nodes", "used_gpus", "used_gpu_milli", "total_gpus", "arrived_gpu_milli", "used_cpu_milli",
               "arrived_cpu_milli"]


@pytest.mark.parametrize("name,pol,sel", POLICIES[:2] + POLICIES[4:5], ids=["FGD", "BestFit", "GpuClustering"])
def test_fuzz_cluster_report(case, name, pol, sel):
    # the per-event cluster report (analysis.go:59-119) on every path: the oracle's exact sums
    want_res, _, want = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=pol, gpu_sel=sel,
                                     seed=5, threads=16, with_report=True)
    for mode, label in PATHS:
        eng = ksim.Engine(len(case["onodes"]), 1, run_mode=mode)
        try:
            eng.set_nodes(0, case["nodes"])
            eng.set_typical(0, case["typical"], case["typical_n"])
            eng.set_policy(0, name, seed=5)
            eng.set_report(True)
            eng.load_events(0, case["events"], case["n_events"])
            eng.run()
            assert eng.results(0) == want_res, label
            got = eng.reports(0)
        finally:
            eng.close()
        assert len(got) == len(want)
        for i, (g, w) in enumerate(zip(got, want)):
            assert g["frag_bins"] == w["frag_bins_exact"], (label, i)
            assert [g[k] for k in REPORT_KEYS] == [w[k] for k in REPORT_KEYS], (label, i)


@pytest.mark.parametrize("world", [2, 3, 5])
@pytest.mark.parametrize("name,pol,sel", POLICIES, ids=[p[0] for p in POLICIES])
def test_fuzz_node_sharded_group(case, world, name, pol, sel):
    # one cluster split over `world` shard engines (in-process group, the multi-GPU exchange's protocol)
    import ksim.shard as SH
    n = len(case["onodes"])
    if n < world:
        pytest.skip("fewer nodes than shards")
    want, _, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=pol, gpu_sel=sel, seed=5,
                              threads=16)
    g = SH.ShardGroup(case["nodes"], (case["typical"], case["typical_n"]), world, policy=name, seed=5)
    try:
        g.load_events(case["events"], case["n_events"])
        g.run()
        got = g.results()
    finally:
        g.close()
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, "first mismatch at %d: %s vs %s" % (bad[0], got[bad[0]], want[bad[0]])


def test_fuzz_multi_replica_mixed_policies():
    # six replicas of one node set, one per policy, ragged event streams from different seeds, one run
    cases = [make_case(20 + r, 150, 300 + 150 * r, 0.2) for r in range(len(POLICIES))]
    eng = ksim.Engine(150, len(POLICIES))
    try:
        for r, (name, _, _) in enumerate(POLICIES):
            eng.set_nodes(r, cases[r]["nodes"])
            eng.set_typical(r, cases[r]["typical"], cases[r]["typical_n"])
            eng.set_policy(r, name, seed=5)
            eng.load_events(r, cases[r]["events"], cases[r]["n_events"])
        eng.run()
        for r, (name, pol, sel) in enumerate(POLICIES):
            c = cases[r]
            want, want_state, _ = O.run_events(c["onodes"], c["otypical"], c["oevents"], policy=pol, gpu_sel=sel,
                                               seed=5, threads=16)
            assert eng.results(r) == want, name
            check_state(eng.nodes(r), want_state)
    finally:
        eng.close()


@pytest.mark.parametrize("policy", ["PWR", "PWR 500 FGD 500", "PWR 100 FGD 900"])
@pytest.mark.parametrize("seed,n,e,pdel", [(31, 60, 700, 0.2), (32, 300, 1200, 0.0)])
def test_fuzz_pwr(policy, seed, n, e, pdel):
    # PWRScore and the weighted PWR + FGD sums (k_step + k_step_pwr), on the openb model vocabulary
    # so that the reference's energy tables (const.go:41-124) apply
    t = ksim.Trace.openb("default")
    c = make_case(seed, n, e, pdel, models=t.type_names())
    name, w = ksim.parse_policy(policy)
    pol, sel = (O.POL_PWR, O.SEL_PWR) if name == "PWR" and not w else (O.POL_PWR_FGD, O.SEL_FGD)
    w_pwr, w_fgd = w if w else (0, 0)
    want, want_state, _ = O.run_events(c["onodes"], c["otypical"], c["oevents"], policy=pol, gpu_sel=sel,
                                       threads=16, w_pwr=w_pwr, w_fgd=w_fgd)
    eng = ksim.Engine(n, 1)
    try:
        eng.set_nodes(0, c["nodes"])
        eng.set_typical(0, c["typical"], c["typical_n"])
        eng.set_policy(0, policy)
        eng.set_power_model(0, t.power_model())
        eng.load_events(0, c["events"], c["n_events"])
        eng.run()
        got, state = eng.results(0), eng.nodes(0)
    finally:
        eng.close()
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, "first mismatch at %d: %s vs %s" % (bad[0], got[bad[0]], want[bad[0]])
    check_state(state, want_state)


@pytest.mark.parametrize("name,pol,sel", POLICIES[1:], ids=[p[0] for p in POLICIES[1:]])
def test_fuzz_scan1_records_in_lds(name, pol, sel):
    # one workgroup per replica on a cluster past the VGPR form's 1280 nodes: k_scan1 with the node
    # records in LDS (the record placement k_scan1 picks above 1280 nodes)
    case = make_case(11, 2000, 1500)
    want, want_state, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=pol, gpu_sel=sel,
                                       seed=5, threads=16)
    eng = ksim.Engine(2000, 1, wgs_per_replica=1)
    try:
        eng.set_nodes(0, case["nodes"])
        eng.set_typical(0, case["typical"], case["typical_n"])
        eng.set_policy(0, name, seed=5)
        eng.load_events(0, case["events"], case["n_events"])
        eng.run()
        got, state = eng.results(0), eng.nodes(0)
        assert eng.last_run_path() == "k_scan1"
    finally:
        eng.close()
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert len(got) == len(want) and not bad, "first mismatch at event %d" % bad[0]
    check_state(state, want_state)
