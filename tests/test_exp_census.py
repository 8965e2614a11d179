"""math.Exp on the FGD path is pinned.

The FGD score is int64(sigmoid((cur - new) / 1000) * 100) (fgd_score.go:123,144, plugin_utils.go:76-78);
the product and the oracle restate Go's portable exp (src/math/exp.go), while the reference binary
may have linked another exp routine.  tests/golden/make_exp_census.py replayed all 170 FGD
experiments of the paper sweep through the oracle and recorded every score delta that reaches the
sigmoid.  The committed census says:
  - on every delta within 1e-10 of a step of the score function (1.2e8 of 2.4e9), the portable exp
    and a correctly rounded exp give the same score (crdiff 0), and the whole decision stream of every
    experiment is unchanged when the oracle uses the correctly rounded exp;
  - the deltas whose score an exp error of one ulp WOULD flip all have |delta| <= 4.6e-13, i.e. an exp
    argument |x| <= 4.6e-16, far inside Go's NearZero branch (|x| < 2^-28: exp = 1 + x, the correctly
    rounded value).  So any exp that is correctly rounded there -- every accurate implementation --
    reproduces the reference's decisions on these traces.
This file checks the golden summary and re-runs the census on its bounded prefix sample live.
"""
import json
import os

import pytest

import helpers
import ksim
import pyoracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "exp_census.json")


@pytest.fixture(scope="module")
def census():
    with open(GOLDEN) as f:
        return json.load(f)


def test_summary_pins_exp(census):
    s = census["summary"]
    assert s["experiments"] == 170  # 17 traces x seeds 42..51, FGD
    assert s["deltas"] > 2e9 and s["near"] > 1e8
    assert s["crdiff"] == 0
    assert s["all_same_decisions_cr"]
    # every exp-sensitive delta sits in Go's NearZero branch (|x| = |delta| / 1000 < 2^-28)
    assert s["sensitive_max_abs_delta"] / 1000.0 < 2.0 ** -28
    for name, c in census["experiments"].items():
        assert c["crdiff"] == 0 and c["same_decisions_cr"], name
        assert c["crdiff_cases"] == [], name


def test_thresholds_match_the_oracle(census):
    assert O.score_thresholds()[1:101] == census["thresholds"]


def test_ulp_nudges_are_a_real_hazard(census):
    # an exp that is off by one ulp everywhere WOULD change decisions: the census is not vacuous
    c = census["experiments"]["openb_pod_list_default/06-FGD/42"]
    assert c["decisions_changed_nudge+1"] > 0 and c["decisions_changed_nudge-1"] > 0


def test_prefix_census_live(census):
    # the bounded sample (default trace, seed 42, first 1500 events) re-run on the oracle
    want = census["prefix"]
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=42, tune_ratio=1.3, shuffle=True)
    args = (helpers.oracle_nodes(t, rp), helpers.oracle_typical(t), helpers.oracle_events(t, rp, want["events"]))
    O.census_begin()
    base, _, _ = O.run_events(*args, threads=8)
    got = O.census_end()
    for k in ("deltas", "near", "crdiff", "sensitive", "min_dist", "sensitive_max_abs_delta"):
        assert got[k] == want[k], k
    O.set_exp_mode(1)
    try:
        cr, _, _ = O.run_events(*args, threads=8)
    finally:
        O.set_exp_mode(0)
    assert cr == base


def test_replay_cache_steps_aside_for_oracle_state(monkeypatch):
    # a replay under a census, a nudged exp or the correctly rounded exp must run, never come
    # from the cache a default-state replay of the same arguments filled
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=43, tune_ratio=1.3, shuffle=True)
    args = (helpers.oracle_nodes(t, rp)[:40], helpers.oracle_typical(t), helpers.oracle_events(t, rp, 60))
    calls = []
    real = O._run_events

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)
    monkeypatch.setattr(O, "_run_events", counting)
    monkeypatch.setenv("KSIM_ORACLE_CACHE", "1")
    base = O.run_events(*args)
    n0 = len(calls)
    assert O.run_events(*args) == base and len(calls) == n0          # default state: served from the cache
    for enter, leave in ((lambda: O.set_exp_mode(1), lambda: O.set_exp_mode(0)),
                         (lambda: O.set_exp_nudge(1), lambda: O.set_exp_nudge(0)),
                         (O.census_begin, O.census_end)):
        enter()
        try:
            before = len(calls)
            O.run_events(*args)
            assert len(calls) == before + 1
        finally:
            leave()
    before = len(calls)
    assert O.run_events(*args) == base and len(calls) == before      # back to the default: cached again
