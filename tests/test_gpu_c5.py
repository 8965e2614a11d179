"""C5: the synthetic 100k-node / 1M-pod cluster on one MI355X.

The default path is the wide k_hmemo (63 workgroups, each owning 1600 ranks: their records and the
L1 of their (class, node) keys in LDS, the keys in HBM; one exchange per pod).  k_replay (run_mode
2) spreads the replica over 256 workgroups of ~391 LDS-resident nodes and re-scores every node per
pod.  Parity: the first events bit-exact against the oracle on all 100k nodes on both; k_hmemo,
k_replay and the independent k_step path equal on a longer prefix; over the full 1M-event replay
k_hmemo equals k_replay, and size-independent properties hold (the final cluster state equals the
host-side replay of the reported binds, no GPU over-committed).
"""
import numpy as np
import pytest

import helpers
import ksim
import pyoracle as O

pytestmark = pytest.mark.gpu

N_NODES, N_PODS = 100_000, 1_000_000


@pytest.fixture(scope="module")
def c5():
    base = ksim.Trace.openb("default")
    t = base.synthetic(N_NODES, N_PODS, seed=0)
    rp = t.replay(seed=1, tune_ratio=0.0, shuffle=False)
    return t, rp


def run(t, rp, n_ev, run_mode=0, wgs=0, policy="FGD"):
    arr, n = t.typical()
    eng = ksim.Engine(t.num_nodes, 1, run_mode=run_mode, wgs_per_replica=wgs)
    eng.set_nodes(0, rp.nodes)
    eng.set_typical(0, arr, n)
    eng.set_policy(0, policy)
    eng.load_events(0, rp.events, n_ev)
    ms = eng.run()
    out = (eng.results(0), eng.nodes(0), ms, eng.last_run_wgs())
    eng.close()
    return out


@pytest.mark.parametrize("run_mode", [0, 2], ids=["hmemo", "replay"])
def test_c5_prefix_vs_oracle(c5, run_mode):
    # auto: the wide k_hmemo (63 workgroups of 1600 ranks); run_mode 2: k_replay over 256 workgroups
    t, rp = c5
    n_ev = 300
    res, state, _, k = run(t, rp, n_ev, run_mode=run_mode)
    assert k > 64 if run_mode == 2 else k == 63  # k_replay's wide (4 granule columns per polling lane) exchange
    want, want_state, _ = O.run_events(helpers.oracle_nodes(t, rp), helpers.oracle_typical(t),
                                       helpers.oracle_events(t, rp, n_ev), policy=O.POL_FGD, gpu_sel=O.SEL_FGD,
                                       threads=16)
    assert res == want


def test_c5_replay_vs_step_kernel(c5):
    t, rp = c5
    n_ev = 2500
    a, sa, _, _ = run(t, rp, n_ev)
    b, sb, _, _ = run(t, rp, n_ev, run_mode=1)
    c, sc, _, _ = run(t, rp, n_ev, run_mode=2)
    assert a == b == c
    assert bytes(sa) == bytes(sb) == bytes(sc)


def test_c5_full_replay_properties(c5):
    t, rp = c5
    res, state, ms, k = run(t, rp, rp.n)
    assert len(res) == N_PODS
    st = np.array([r[4] for r in res])
    assert set(np.unique(st)) <= {ksim.SCHEDULED, ksim.UNSCHEDULABLE}
    sched = st == ksim.SCHEDULED
    assert 0.3 < sched.mean() < 0.95  # ~146% GPU demand: the cluster fills, then pods fail
    # host replay of the reported binds reproduces the device's final state
    nodes = rp.nodes
    cpu = np.array([nodes[i].cpu_alloc_milli for i in range(N_NODES)], dtype=np.int64)
    gpu_used = np.zeros((N_NODES, 8), dtype=np.int64)
    cpu_used = np.zeros(N_NODES, dtype=np.int64)
    ev = rp.events
    for i in np.nonzero(sched)[0]:
        node, mask = res[i][0], res[i][1]
        cpu_used[node] += ev[i].cpu_milli
        for g in range(8):
            if mask >> g & 1:
                gpu_used[node, g] += ev[i].gpu_milli
    for i in range(0, N_NODES, 7):
        s = state[i]
        assert s.cpu_used_milli == cpu_used[i]
        assert list(s.gpu_used_milli) == list(gpu_used[i])
    assert (gpu_used <= 1000).all() and (cpu_used <= cpu).all()
    # the scanning k_replay (256 workgroups) reaches the same 1M decisions
    res2, _, ms2, k2 = run(t, rp, rp.n, run_mode=2)
    assert res2 == res
    print("C5 FGD: %d events on %d nodes: k_hmemo (%d workgroups) %.1f ms, k_replay (%d) %.1f ms"
          % (N_PODS, N_NODES, k, ms, k2, ms2))


@pytest.mark.parametrize("world", [2, 8])
def test_c5_sharded_group_equals_unsharded(c5, world):
    # the node-sharded mode at C5 scale, as an in-process group on one device (the
    # same per-shard kernels as one process per GPU; the exchange is a gather kernel, not RCCL)
    import time
    import ksim.shard as SH
    t, rp = c5
    n_ev = 5000
    want, _, ms1, _ = run(t, rp, n_ev, run_mode=2)
    g = SH.ShardGroup(rp.nodes, t.typical(), world)
    try:
        g.load_events(rp.events, n_ev)
        t0 = time.perf_counter()
        ms = g.run()
        wall = time.perf_counter() - t0
        assert g.results() == want
    finally:
        g.close()
    print("C5 %d events: unsharded k_replay %.1f us/pod, %d-shard group %.1f us/pod (wall %.1f)"
          % (n_ev, ms1 * 1e3 / n_ev, world, ms * 1e3 / n_ev, wall * 1e6 / n_ev))


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("policy", ["BestFit", "GpuPacking", "DotProd", "GpuClustering", "Random"])
def test_c5_sharded_cheap_policies_on_replay_slices(c5, world, policy):
    # round-5 verdict item 7: the other policies' node-sharded group on k_replay slices -- every shard's slices in
    # ONE launch and one granule exchange per pod over all of them (BestFit's NormalizeScore range in the same
    # granules), instead of r02's per-pod k_step + gather + commit launches: equal to the unsharded run on 5 000
    # events, and timed per pod
    import time
    import ksim.shard as SH
    t, rp = c5
    n_ev = 5000
    want, _, ms1, _ = run(t, rp, n_ev, run_mode=2, policy=policy)
    g = SH.ShardGroup(rp.nodes, t.typical(), world, policy=policy)
    try:
        g.load_events(rp.events, n_ev)
        t0 = time.perf_counter()
        ms = g.run()
        wall = time.perf_counter() - t0
        assert g.engines[0].last_run_kernels() == ["k_replay_group"]
        assert g.results() == want
    finally:
        g.close()
    print("C5 %s %d events: unsharded k_replay %.1f us/pod, %d-shard k_replay group %.2f us/pod (wall %.1f)"
          % (policy, n_ev, ms1 * 1e3 / n_ev, world, ms * 1e3 / n_ev, wall * 1e6 / n_ev))
