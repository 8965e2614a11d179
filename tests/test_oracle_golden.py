"""The oracle against the reference's own Go known answers (tests/golden/go_known_answers.json)."""
import ctypes as C
import json
import math
import os
from fractions import Fraction

import pytest

import pyoracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "go_known_answers.json")))


def tp_of(name):
    rows = GOLD[name]
    return O.typical([(r["cpu"], r["milli"], r["num"], r["type"], float(Fraction(*r["pct"]))) for r in rows])


def node_of(d):
    return O.node_res(d["cpu_left"], d["gpu_left"], d["gpu_number"], d["type"], d["cpu_cap"])


def pod_of(d):
    return O.pod_res(d["cpu"], d["milli"], d["num"], d["type"])


@pytest.mark.parametrize("case", GOLD["frag_score_cases"], ids=lambda c: c["src"])
def test_frag_amount_score(case):
    # frag_test.go: assert.InDelta(want, score, 0.01)
    tp = tp_of(case["typical"])
    n = node_of(case["node"])
    got = O.frag_score(n, tp)
    assert abs(got - case["want"]) <= 0.01
    # NodeGpuShareFragAmount(...).FragAmountSumExceptQ3() is the same number
    bins = O.frag_bins(n, tp)
    assert sum(b for i, b in enumerate(bins) if i != O.Q3) == pytest.approx(got, rel=1e-12)
    if "want_class" in case:
        L = O.lib()
        p = O.pod_res(*(lambda r: (r["cpu"], r["milli"], r["num"], r["type"]))(GOLD[case["typical"]][0]))
        assert L.orc_get_node_pod_frag(C.byref(n), C.byref(p)) == O.Q4
        assert L.orc_get_gpu_milli_left_total(C.byref(n)) == case["want_left_total"]


@pytest.mark.parametrize("case", GOLD["frag_milli_cases"])
def test_gpu_frag_milli(case):
    assert O.lib().orc_get_gpu_frag_milli(C.byref(node_of(case["node"])), C.byref(pod_of(case["pod"]))) == case["want"]


@pytest.mark.parametrize("case", GOLD["packing_cases"])
def test_packing_score(case):
    n = node_of(case["node"])
    before = list(n.milli_gpu_left)[: n.n_gpu_left]
    err = C.c_int(0)
    assert O.lib().orc_packing_score(C.byref(n), C.byref(pod_of(case["pod"])), C.byref(err)) == case["want"]
    assert err.value == 0
    assert list(n.milli_gpu_left)[: n.n_gpu_left] == before  # order of MilliGpuLeftList unchanged


@pytest.mark.parametrize("case", GOLD["flatten_cases"])
def test_flatten(case):
    buf = C.create_string_buffer(256)
    O.lib().orc_flatten_milli_gpu(C.byref(node_of(case["node"])), buf, 256)
    assert buf.value.decode() == case["want"]


@pytest.mark.parametrize("case", GOLD["add_cases"])
def test_add(case):
    out = O.NodeResource()
    idl = (C.c_int * len(case["idl"]))(*case["idl"])
    rc = O.lib().orc_node_add(C.byref(node_of(case["node"])), C.byref(pod_of(case["pod"])), idl, len(case["idl"]),
                              C.byref(out))
    assert rc == 0
    assert out.milli_cpu_left == case["want_cpu_left"]
    assert list(out.milli_gpu_left)[: out.n_gpu_left] == case["want_gpu_left"]


@pytest.mark.parametrize("case", GOLD["sub_cases"])
def test_sub(case):
    out = O.NodeResource()
    rc = O.lib().orc_node_sub(C.byref(node_of(case["node"])), C.byref(pod_of(case["pod"])), C.byref(out))
    assert rc == 0
    assert out.milli_cpu_left == case["want_cpu_left"]
    assert list(out.milli_gpu_left)[: out.n_gpu_left] == case["want_gpu_left"]


def test_go_exp_matches_libm_closely():
    # Go's portable exp is < 1 ulp; it must agree with glibc to within 1 ulp on the sigmoid range.
    L = O.lib()
    import random
    rnd = random.Random(0)
    for _ in range(20000):
        x = rnd.uniform(-40, 40)
        a, b = L.orc_go_exp(x), math.exp(x)
        assert abs(a - b) <= 1.0 * math.ulp(b)
    for x in (0.0, -0.0, 1e-30, -1e-30, 3.7252902984e-09):
        assert L.orc_go_exp(x) == 1 + x
    assert L.orc_go_exp(800.0) == math.inf and L.orc_go_exp(-800.0) == 0.0


def test_fgd_score_share_pod_picks_first_best_gpu():
    # fgd_score.go:111-133: candidate per GPU with enough milli; first index on ties
    tp = tp_of("typical_35")
    n = O.node_res(32000, [1000, 1000, 1000, 1000], 4, "T4", 64000)
    s, mask = O.fgd_score(n, O.pod_res(4000, 500, 1, ""), tp)
    assert 0 <= s <= 100 and mask == 1  # all GPUs identical -> GPU 0
    n2 = O.node_res(32000, [1000, 300, 1000, 600], 4, "T4", 64000)
    s2, mask2 = O.fgd_score(n2, O.pod_res(4000, 500, 1, ""), tp)
    assert mask2 in (1, 2, 4, 8) and (mask2 & 0b0010) == 0  # GPU 1 cannot fit 500


def test_typical_pods_threshold_and_renorm():
    # frag.go:285-380: top specs until cumulative >= threshold, freq renormalised to sum 1
    wl = [(1000, 0, 0, "")] * 50 + [(2000, 500, 1, "")] * 30 + [(4000, 1000, 1, "")] * 15 + [(8000, 1000, 2, "")] * 5
    tp = O.get_typical_pods(wl, threshold=90, step=1)
    assert [(c, m, n) for (c, m, n, _, _) in tp] == [(1000, 0, 0), (2000, 500, 1), (4000, 1000, 1)]
    assert tp[0][4] == (50 / 100) / (95 / 100)
    assert abs(sum(x[4] for x in tp) - 1) < 1e-12
    # ties in count: reverse Less -> larger MilliCpu first
    wl2 = [(1000, 0, 0, "")] * 10 + [(3000, 0, 0, "")] * 10
    tp2 = O.get_typical_pods(wl2, threshold=100, step=1)
    assert [x[0] for x in tp2] == [3000, 1000]


def test_report_exact_sum_is_fsum():
    # The oracle's exact cluster bins (fixed point 2^-80, orc_fix80) equal math.fsum of the
    # per-node NodeGpuShareFragAmount bins (correctly rounded sum), at several prefixes of a run.
    import math
    import ksim
    import helpers
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=42)
    keep = list(range(0, t.num_nodes, 5))
    onodes = helpers.oracle_subset(t, rp, keep)
    tl = helpers.oracle_typical(t)
    tp = O.typical(tl)
    for n_ev in (1, 200, 900):
        res, state, reps = O.run_events(onodes, tl, helpers.oracle_events(t, rp, n_ev), threads=8,
                                        with_report=True)
        per_node = []
        for d, (cpu_left, _, _, gl) in zip(onodes, state):
            nr = O.node_res(cpu_left, gl[:d["gpu"]], d["gpu"], d["model"], d["cpu"])
            per_node.append(O.frag_bins(nr, tp))
        exact = [math.fsum(b[k] for b in per_node) for k in range(7)]
        assert reps[-1]["frag_bins_exact"] == exact
        for a, b in zip(reps[-1]["frag_bins"], exact):
            assert abs(a - b) <= 1e-12 * max(b, 1.0)


def test_oracle_rejects_bad_deletions():
    # a deletion must name an earlier creation, at most once (mirrors ksim_engine_load_events)
    nodes = [dict(name="n0", cpu=8000, mem=8192, pods=110, gpu=1, model="T4")]
    tp = [(1000, 0, 0, "", 1.0)]
    pod = dict(cpu=1000, mem=100, milli=0, num=0, type="")
    for evs in ([pod, dict(pod, delete=1, ref=0), dict(pod, delete=1, ref=0)],
                [pod, dict(pod, delete=1, ref=0), dict(pod, delete=1, ref=1)]):
        with pytest.raises(AssertionError):
            O.run_events(nodes, tp, evs)
    O.run_events(nodes, tp, [pod, dict(pod, delete=1, ref=0)])  # a valid stream runs


@pytest.mark.parametrize("case", GOLD["dot_product_cases"])
def test_dot_product_vectors(case):
    # utils_test.go:25-55: NormalizeVector then CalculateVectorDotProduct, InDelta 1e-3 as the Go test
    nv = O.normalize_vector(case["node_vec"], case["cap"])
    pv = O.normalize_vector(case["pod_vec"], case["cap"])
    assert abs(O.vector_dot_product(nv, pv) - case["want"]) <= 1e-3


def test_dot_product_vector_edges():
    # CalculateVectorDotProduct: -1 on empty or unequal vectors; NormalizeVector: 0 where the norm is
    # not positive, the input unchanged when the lengths differ
    assert O.vector_dot_product([], [1.0]) == -1 and O.vector_dot_product([1.0, 2.0], [1.0]) == -1
    assert O.normalize_vector([3.0, 4.0], [0.0, 2.0]) == [0.0, 2.0]
    assert O.normalize_vector([3.0, 4.0], [2.0]) == [3.0, 4.0]


def test_dot_product_variants_reference_examples():
    # config.go:8-28 worked example: pod <100 CPU, 100 GPU>, node <3000 CPU, GPUs 200, 500, 1000 x 6>
    n = O.node_res(3000, [200, 500] + [1000] * 6, 8, "", 3000)
    p = O.pod_res(100, 100, 1, "")
    # share: virtual nodes <3000, 200>, <3000, 500>, <3000, 6000>; divide scales the CPU by GPU share
    for dim in (O.DIM_SHARE, O.DIM_DIVIDE, O.DIM_EXTEND):
        for norm in (O.NORM_MAX, O.NORM_NODE, O.NORM_POD):
            s, g = O.dot_product_score(n, p, dim, norm)
            assert 0 <= s <= 100 and g in (1, 2, 4)  # a share GPU (0 or 1) or the first idle GPU (2)
    # merge has no GPU id: the DotProduct selector cannot place a GPU pod with it
    assert O.dot_product_score(n, p, O.DIM_MERGE, O.NORM_MAX)[1] == 0
