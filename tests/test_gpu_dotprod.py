"""GPU parity of DotProductScore under every GpuPluginCfg (pkg/type/config.go:3-55): dimExtMethod merge /
share / divide / extend x normMethod max / node / pod, with Open-Gpu-Share's gpuSelMethod "best" and
"DotProductScore" (allocateGpuIdBasedOnDotProduct, dot_product_score.go:102-107; the reference's harness
switches to it whenever dimExtMethod is not merge, generate_config_and_run.py:271-275).

Bar: bit-exact (node, GPU set, score, feasible count, status) per event against the oracle's literal
restatement of GenerateSchedulingMatchGroups (oracle/fgd_oracle.c), and the same final cluster state, on
k_replay (auto K and K = 1), the per-pod k_step path, a node-sharded group and the adversarial fuzz
clusters.  The reference holds expected results only for merge / max (the paper's configuration,
tests/test_gpu_sweep.py); the other configurations are pinned by the restated formulas and by
utils_test.go's NormalizeVector / CalculateVectorDotProduct vectors (tests/test_oracle_golden.py).
Every test needs a gfx950 device.
"""
import pytest

import helpers
import ksim
import ksim.shard as SH
import pyoracle as O
from fuzz_cases import make_case
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

DIMS = ["merge", "share", "divide", "extend"]
NORMS = ["max", "node", "pod"]
ODIM = {"merge": O.DIM_MERGE, "share": O.DIM_SHARE, "divide": O.DIM_DIVIDE, "extend": O.DIM_EXTEND}
ONORM = {"max": O.NORM_MAX, "node": O.NORM_NODE, "pod": O.NORM_POD}
PATHS = {"k_replay": dict(), "k_scan1-K1": dict(wgs_per_replica=1), "k_step": dict(run_mode=1)}


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def oracle_sel(dim, gpusel):
    if gpusel is None:
        return O.SEL_DOTPROD if dim != "merge" else O.SEL_BEST
    return {"best": O.SEL_BEST, "DotProd": O.SEL_DOTPROD}[gpusel]


def run_engine(nodes, nn, typical, events, n_ev, dim, norm, gpusel=None, report=False, **kw):
    arr, n = typical
    eng = ksim.Engine(nn, 1, **kw)
    try:
        eng.set_nodes(0, nodes)
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "DotProd", gpusel=gpusel, dim_ext=dim, norm=norm)
        if report:
            eng.set_report(True)
        eng.load_events(0, events, n_ev)
        eng.run()
        return eng.results(0), eng.nodes(0), eng.last_run_path()
    finally:
        eng.close()


@pytest.mark.parametrize("norm", NORMS)
@pytest.mark.parametrize("dim", DIMS)
def test_subset_replay(default_trace, dim, norm):
    # one oracle replay per configuration, every execution path against it
    rp = default_trace.replay(seed=42)
    keep = list(range(3, default_trace.num_nodes, 7))  # 173 nodes, every GPU model
    n_ev = 1500
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    want, want_state, _ = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                       helpers.oracle_events(default_trace, rp, n_ev), policy=O.POL_DOTPROD,
                                       gpu_sel=oracle_sel(dim, None), threads=16, dim_ext=ODIM[dim], norm=ONORM[norm])
    for run in sorted(PATHS):
        res, state, path = run_engine(helpers.subset_nodes(rp, keep), len(keep), default_trace.typical(), rp.events,
                                      n_ev, dim, norm, **PATHS[run])
        assert path == run.split("-")[0]
        assert_same(res, want, state, want_state, keep)


@pytest.mark.parametrize("dim", ["share", "extend"])
def test_best_fit_selector_with_split_dims(default_trace, dim):
    # gpuSelMethod "best" given explicitly: the score plugin's configuration, the best-fit GPU choice
    rp = default_trace.replay(seed=43)
    keep = list(range(0, default_trace.num_nodes, 5))
    res, state, _ = run_engine(helpers.subset_nodes(rp, keep), len(keep), default_trace.typical(), rp.events, 2000,
                               dim, "node", gpusel="best")
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    want, want_state, _ = O.run_events(onodes, helpers.oracle_typical(default_trace),
                                       helpers.oracle_events(default_trace, rp, 2000), policy=O.POL_DOTPROD,
                                       gpu_sel=O.SEL_BEST, threads=16, dim_ext=ODIM[dim], norm=O.NORM_NODE)
    assert_same(res, want, state, want_state, keep)


def test_merge_with_dotprod_selector_fails_gpu_pods(default_trace):
    # merge groups carry no GPU id: with gpuSelMethod "DotProductScore" every GPU pod's Reserve fails
    rp = default_trace.replay(seed=44)
    keep = list(range(0, default_trace.num_nodes, 11))
    res, _, _ = run_engine(helpers.subset_nodes(rp, keep), len(keep), default_trace.typical(), rp.events, 300,
                           "merge", "max", gpusel="DotProd")
    ev = rp.events
    assert all(r[4] == ksim.ERROR for i, r in enumerate(res) if ev[i].gpu_milli > 0 and r[3] > 0)


@pytest.mark.parametrize("dim,norm", [("divide", "pod"), ("extend", "node")])
def test_full_trace(default_trace, dim, norm):
    rp = default_trace.replay(seed=45)
    res, state, path = run_engine(rp.nodes, default_trace.num_nodes, default_trace.typical(), rp.events, rp.n, dim,
                                  norm)
    assert path == "k_replay"
    want, want_state, _ = O.run_events(helpers.oracle_nodes(default_trace, rp), helpers.oracle_typical(default_trace),
                                       helpers.oracle_events(default_trace, rp), policy=O.POL_DOTPROD,
                                       gpu_sel=O.SEL_DOTPROD, threads=16, dim_ext=ODIM[dim], norm=ONORM[norm])
    assert_same(res, want, state, want_state, None)


@pytest.mark.parametrize("seed,n,e,pdel", [(2, 97, 900, 0.25), (3, 250, 1200, 0.1), (4, 7, 300, 0.4)])
@pytest.mark.parametrize("dim", ["share", "divide", "extend"])
def test_fuzz_clusters(seed, n, e, pdel, dim):
    # adversarial synthetic clusters (3-7 GPU nodes, GPU-less nodes, deletions) on every path
    case = make_case(seed, n, e, pdel)
    for norm in NORMS:
        want, want_state, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=O.POL_DOTPROD,
                                           gpu_sel=O.SEL_DOTPROD, threads=16, dim_ext=ODIM[dim], norm=ONORM[norm])
        for run, kw in sorted(PATHS.items()):
            got, state, _ = run_engine(case["nodes"], n, (case["typical"], case["typical_n"]), case["events"],
                                       case["n_events"], dim, norm, **kw)
            bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
            assert len(got) == len(want) and not bad, "%s/%s/%s: first mismatch at %d: %s vs %s" % (
                dim, norm, run, bad[0], got[bad[0]], want[bad[0]])


@pytest.mark.parametrize("world", [2, 5])
def test_sharded_group(default_trace, world):
    rp = default_trace.replay(seed=46)
    keep = list(range(2, default_trace.num_nodes, 6))
    nodes = helpers.subset_nodes(rp, keep)
    unsh, _, _ = run_engine(nodes, len(keep), default_trace.typical(), rp.events, 1200, "extend", "pod")
    arr, n = default_trace.typical()
    g = SH.ShardGroup(nodes, (arr, n), world, policy="DotProd")
    try:
        for e in g.engines:
            e.set_policy(0, "DotProd", dim_ext="extend", norm="pod")
        g.load_events(rp.events, 1200)
        g.run()
        assert g.results() == unsh
    finally:
        g.close()


def test_report_matches_k_step(default_trace):
    rp = default_trace.replay(seed=47)
    keep = list(range(1, default_trace.num_nodes, 4))
    arr, n = default_trace.typical()
    reps = {}
    for run, kw in (("k_replay", {}), ("k_step", dict(run_mode=1))):
        eng = ksim.Engine(len(keep), 1, **kw)
        eng.set_nodes(0, helpers.subset_nodes(rp, keep))
        eng.set_typical(0, arr, n)
        eng.set_policy(0, "DotProd", dim_ext="share", norm="pod")
        eng.set_report(True)
        eng.load_events(0, rp.events, 2500)
        eng.run()
        reps[run] = (eng.results(0), eng.reports(0))
        eng.close()
    assert reps["k_replay"] == reps["k_step"]


def test_plugin_cfg_errors():
    eng = ksim.Engine(4, 1)
    try:
        with pytest.raises(KeyError):
            eng.set_policy(0, "DotProd", dim_ext="bogus")
        with pytest.raises(ksim.KsimError) as ei:
            eng.set_policy(0, "BestFit", gpusel="DotProd")  # allocateGpuIdFunc has no DotProductScore entry
        assert ei.value.code == ksim.KSIM_ENOTSUP
        from ksim import lib
        assert lib().ksim_engine_set_plugin_cfg(eng.h, 0, 4, 0) == ksim.KSIM_ENOTSUP
        assert lib().ksim_engine_set_plugin_cfg(eng.h, 0, 0, 3) == ksim.KSIM_ENOTSUP
    finally:
        eng.close()
