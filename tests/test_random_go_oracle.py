"""The oracle's Random draw structure on Go's math/rand stream (fgd_oracle.c, orc_policy.go_stream)
against a pure-Python restatement on small clusters: per creation event scheduler.go:464 Intn(100),
default_preemption.go:183 Int31n(#nodes) when nothing fits, random_score.go:44 Intn(#feasible) over
the feasible list in node order when two or more fit, and the random GPU selector's Intn(k) per
fitting GPU (open_gpu_share.go:325-343).  The draws come from the oracle's Go source, itself pinned
to Go's published outputs (tests/test_go_rand.py); the Filter here is the plain resource fit of
these untyped pods.  CPU only."""
import random

import pytest

import pyoracle as O


def py_random_go(nodes, events, seed, gpusel):
    g = O.go_seed(seed)
    cpu = [0] * len(nodes)
    mem = [0] * len(nodes)
    pods = [0] * len(nodes)
    gl = [[1000] * n["gpu"] for n in nodes]
    out = []
    for e in events:
        O.go_int31n(g, 100)
        feas = []
        for i, n in enumerate(nodes):
            ok = cpu[i] + e["cpu"] <= n["cpu"] and mem[i] + e["mem"] <= n["mem"] and pods[i] + 1 <= n["pods"]
            if ok and e["milli"] > 0:
                if e["milli"] < 1000:
                    ok = any(v >= e["milli"] for v in gl[i])
                else:
                    ok = sum(1 for v in gl[i] if v == 1000) >= e["num"]
            if ok:
                feas.append(i)
        if not feas:
            O.go_int31n(g, len(nodes))
            out.append((-1, 0, 0, 0, 1))
            continue
        k = 0 if len(feas) == 1 else O.go_int31n(g, len(feas))
        node = feas[k]
        mask = 0
        if 0 < e["milli"] < 1000:
            if gpusel == O.SEL_RANDOM:
                c = 0
                for gi, v in enumerate(gl[node]):
                    if v >= e["milli"]:
                        c += 1
                        if O.go_int31n(g, c) == 0:
                            mask = 1 << gi
            else:  # best fit: the fitting GPU with the least milli left, first index on ties
                best = min((v, gi) for gi, v in enumerate(gl[node]) if v >= e["milli"])
                mask = 1 << best[1]
        elif e["milli"] == 1000:
            free = [gi for gi, v in enumerate(gl[node]) if v == 1000][: e["num"]]
            mask = sum(1 << gi for gi in free)
        cpu[node] += e["cpu"]
        mem[node] += e["mem"]
        pods[node] += 1
        for gi in range(len(gl[node])):
            if mask >> gi & 1:
                gl[node][gi] -= e["milli"]
        out.append((node, mask, 100000 if len(feas) > 1 else 0, len(feas), 0))
    return out


def small_case(seed, n_nodes, n_ev):
    rnd = random.Random(seed)
    nodes = [dict(name="n%03d" % i, cpu=rnd.choice([8000, 16000, 32000]), mem=rnd.choice([32768, 65536]),
                  pods=rnd.choice([4, 8, 110]), gpu=rnd.choice([0, 1, 2, 4, 8]), model="") for i in range(n_nodes)]
    events = []
    for _ in range(n_ev):
        kind = rnd.random()
        milli, num = (0, 0) if kind < 0.3 else ((rnd.choice([100, 250, 500, 700]), 1) if kind < 0.8
                                                 else (1000, rnd.choice([1, 2, 4])))
        events.append(dict(cpu=rnd.choice([500, 1000, 4000, 8000]), mem=rnd.choice([1024, 4096, 16384]),
                           milli=milli, num=num, type=""))
    return nodes, events


@pytest.mark.parametrize("seed", [1, 2, 3, 42])
@pytest.mark.parametrize("gpusel", [O.SEL_RANDOM, O.SEL_BEST])
def test_oracle_draw_structure_matches_python(seed, gpusel):
    nodes, events = small_case(seed, 23, 400)
    want = py_random_go(nodes, events, seed, gpusel)
    got, _, _ = O.run_events(nodes, [(0, 500, 1, "", 100.0)], events, policy=O.POL_RANDOM, gpu_sel=gpusel,
                             go_stream=O.go_seed(seed))
    assert got == want
    assert any(r[4] == 1 for r in want) and any(r[3] > 1 for r in want)  # failures and real draws


def test_go_stream_is_deterministic_and_not_the_hash_contract():
    nodes, events = small_case(7, 31, 300)
    a, _, _ = O.run_events(nodes, [(0, 500, 1, "", 100.0)], events, policy=O.POL_RANDOM, gpu_sel=O.SEL_RANDOM,
                           go_stream=O.go_seed(9))
    b, _, _ = O.run_events(nodes, [(0, 500, 1, "", 100.0)], events, policy=O.POL_RANDOM, gpu_sel=O.SEL_RANDOM,
                           go_stream=O.go_seed(9))
    h, _, _ = O.run_events(nodes, [(0, 500, 1, "", 100.0)], events, policy=O.POL_RANDOM, gpu_sel=O.SEL_RANDOM,
                           seed=9)
    assert a == b and a != h
