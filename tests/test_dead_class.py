"""The premise of the dead-class skip, checked on the oracle: on a create-only stream,
once an event of a pod class (one distinct request) finds no feasible node, every later event of that
class finds none either -- Filter is monotone in the resources a creation takes.  Every policy, the
openb default trace (the C2 stream) and random synthetic clusters (tests/fuzz_cases.py)."""
import pytest

import helpers
import ksim
import pyoracle as O
from fuzz_cases import make_case

POLS = [(O.POL_FGD, O.SEL_FGD), (O.POL_BESTFIT, O.SEL_BEST), (O.POL_PACKING, O.SEL_BEST), (O.POL_RANDOM, O.SEL_RANDOM)]


def check_dead_classes(events, results):
    dead, skippable = set(), 0
    for e, r in zip(events, results):
        if e.get("delete"):
            continue
        key = (e["cpu"], e["cpu_nz"], e["mem"], e["milli"], e["num"], e["type"])
        if key in dead:
            assert r[0] < 0 and r[3] == 0, "a dead class found a node: %s %s" % (key, r)
            skippable += 1
        if r[3] == 0:  # no feasible node (r = node, mask, score, n_feasible, status)
            dead.add(key)
    return skippable


@pytest.mark.parametrize("pol,sel", POLS)
def test_openb_default_dead_classes(pol, sel):
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=42, tune_ratio=1.3, shuffle=True)
    keep = list(range(0, t.num_nodes, 4))  # a quarter of the cluster: it saturates early
    nodes = [helpers.oracle_nodes(t, rp)[i] for i in keep]
    ev = helpers.oracle_events(t, rp, 6000)
    res, _, _ = O.run_events(nodes, helpers.oracle_typical(t), ev, policy=pol, gpu_sel=sel, seed=3, threads=8)
    assert check_dead_classes(ev, res) > 500


@pytest.mark.parametrize("seed", [1, 3, 6, 11])
def test_fuzz_dead_classes(seed):
    case = make_case(seed, 60, 900)
    for pol, sel in POLS:
        res, _, _ = O.run_events(case["onodes"], case["otypical"], case["oevents"], policy=pol, gpu_sel=sel, seed=2,
                                 threads=8)
        check_dead_classes(case["oevents"], res)
