"""Co-residency of the persistent kernels.

k_replay / k_memo with K > 1 workgroups per replica poll each other's granules every step, so every
workgroup of the launch must be resident at once.  The engine sizes K from the occupancy query times
the CUs it may use (KSIM_CUS caps them: a device shared with another process), launches K > 1 grids
cooperatively (the runtime refuses a grid that cannot be resident), and never waits out a poll
timeout: an oversubscribed request either runs correctly with a smaller K or fails at once.
Every test needs a gfx950 device.
"""
import os
import time

import pytest

import helpers
import ksim
import pyoracle as O
from test_gpu_parity import oracle_run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


@pytest.fixture
def cus(monkeypatch):
    def set_cus(n):
        monkeypatch.setenv("KSIM_CUS", str(n))
    return set_cus


def _engine(trace, keep, seeds, n_ev, policy, run_mode=0, wgs=0):
    arr, n = trace.typical()
    eng = ksim.Engine(len(keep), len(seeds), run_mode=run_mode, wgs_per_replica=wgs)
    rps = []
    for r, s in enumerate(seeds):
        rp = trace.replay(seed=s)
        rps.append(rp)
        eng.set_nodes(r, helpers.subset_nodes(rp, keep))
        eng.set_typical(r, arr, n)
        eng.set_policy(r, policy)
        eng.load_events(r, rp.events, n_ev)
    return eng, rps


@pytest.mark.parametrize("policy,pol,sel", [("BestFit", O.POL_BESTFIT, O.SEL_BEST), ("FGD", O.POL_FGD, O.SEL_FGD)])
def test_oversubscribed_request_runs_with_fewer_workgroups(default_trace, cus, policy, pol, sel):
    # 6 replicas x 16 requested workgroups on 24 usable CUs: k_replay cannot hold 96 co-resident
    # workgroups, runs at a K the device holds, and decides as the oracle does
    cus(24)
    keep = list(range(0, default_trace.num_nodes, 4))
    seeds = [42, 43, 44, 45, 46, 47]
    eng, rps = _engine(default_trace, keep, seeds, 600, policy, run_mode=2, wgs=16)
    try:
        t0 = time.time()
        eng.run()
        assert time.time() - t0 < 30
        assert eng.last_run_wgs() * len(seeds) <= 24
        for r, s in enumerate(seeds):
            want, _, _ = oracle_run(default_trace, rps[r], keep, 600, pol, sel)
            assert eng.results(r) == want, s
    finally:
        eng.close()


def test_auto_k_fits_the_usable_cus(default_trace, cus):
    # auto K on 40 usable CUs for 10 replicas: at most 4 workgroups each, same decisions as K = 1
    cus(40)
    keep = list(range(0, default_trace.num_nodes, 3))
    seeds = list(range(42, 52))
    eng, _ = _engine(default_trace, keep, seeds, 500, "GpuPacking", run_mode=2)
    try:
        eng.run()
        k = eng.last_run_wgs()
        assert 1 <= k <= 4
        got = [eng.results(r) for r in range(len(seeds))]
    finally:
        eng.close()
    eng1, _ = _engine(default_trace, keep, seeds, 500, "GpuPacking", run_mode=2, wgs=1)
    try:
        eng1.run()
        assert [eng1.results(r) for r in range(len(seeds))] == got
    finally:
        eng1.close()


def test_memo_that_cannot_be_resident_refuses_at_once(default_trace, cus):
    # k_memo required (run_mode 3) with 10 replicas x 8 workgroups on 32 usable CUs: refused before the
    # launch (KSIM_ENOTSUP), not after a poll timeout
    cus(32)
    keep = list(range(0, default_trace.num_nodes, 2))
    eng, _ = _engine(default_trace, keep, list(range(42, 52)), 300, "FGD", run_mode=3, wgs=8)
    try:
        t0 = time.time()
        with pytest.raises(ksim.KsimError) as ei:
            eng.run()
        assert ei.value.code == ksim.KSIM_ENOTSUP
        assert time.time() - t0 < 10
    finally:
        eng.close()


def test_memo_auto_falls_back_when_not_resident(default_trace, cus):
    # auto mode, same request: k_memo does not fit the usable CUs, the FGD replicas take k_hmemo (one
    # workgroup per replica, no co-residency needed) and match the oracle
    cus(32)
    keep = list(range(0, default_trace.num_nodes, 2))
    seeds = list(range(42, 52))
    eng, rps = _engine(default_trace, keep, seeds, 300, "FGD", run_mode=0, wgs=8)
    try:
        eng.run()
        assert eng.last_run_path() == "k_hmemo"
        for r in (0, 9):
            want, _, _ = oracle_run(default_trace, rps[r], keep, 300, O.POL_FGD, O.SEL_FGD)
            assert eng.results(r) == want
    finally:
        eng.close()
