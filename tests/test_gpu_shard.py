"""Node-sharded single cluster on the GPU: the shards' merged decisions equal the
unsharded engine's (= the oracle's, tests/test_gpu_parity.py) for any number of shards.

The in-process group (ksim_shard_group_run) runs `world` shard engines in lockstep on one device
with the same kernels as the multi-GPU mode; only the exchange differs (one gather kernel instead
of ncclAllGather).  The RCCL exchange itself is exercised at world 1 (a GPU box has one device).
Every test needs a gfx950 device.
"""
import pytest

import helpers
import ksim
import ksim.shard as SH
import pyoracle as O

pytestmark = pytest.mark.gpu

POLICIES = [("FGD", O.POL_FGD, O.SEL_FGD), ("BestFit", O.POL_BESTFIT, O.SEL_BEST),
            ("DotProd", O.POL_DOTPROD, O.SEL_BEST), ("GpuPacking", O.POL_PACKING, O.SEL_BEST),
            ("GpuClustering", O.POL_CLUSTERING, O.SEL_BEST), ("Random", O.POL_RANDOM, O.SEL_RANDOM)]


@pytest.fixture(scope="module")
def default_trace():
    return ksim.Trace.openb("default")


def unsharded(trace, nodes, events, n_ev, policy, seed=0):
    arr, n = trace.typical()
    e = ksim.Engine(len(nodes), 1)
    e.set_nodes(0, nodes)
    e.set_typical(0, arr, n)
    e.set_policy(0, policy, seed=seed)
    e.load_events(0, events, n_ev)
    e.run()
    out = e.results(0)
    e.close()
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_group_fgd_equals_unsharded(default_trace, world):
    rp = default_trace.replay(seed=42)
    n_ev = 1500
    g = SH.ShardGroup(rp.nodes, default_trace.typical(), world)
    g.load_events(rp.events, n_ev)
    g.run()
    got = g.results()
    g.close()
    assert got == unsharded(default_trace, rp.nodes, rp.events, n_ev, "FGD")


@pytest.mark.parametrize("name,pol,sel", POLICIES, ids=[p[0] for p in POLICIES])
def test_group_all_policies_vs_oracle(default_trace, name, pol, sel):
    rp = default_trace.replay(seed=7)
    keep = list(range(1, default_trace.num_nodes, 5))
    nodes = helpers.subset_nodes(rp, keep)
    n_ev = 1200
    g = SH.ShardGroup(nodes, default_trace.typical(), 4, policy=name, seed=3)
    g.load_events(rp.events, n_ev)
    g.run()
    got = g.results()
    g.close()
    onodes = [helpers.oracle_nodes(default_trace, rp)[i] for i in keep]
    want, _, _ = O.run_events(onodes, helpers.oracle_typical(default_trace),
                              helpers.oracle_events(default_trace, rp, n_ev), policy=pol, gpu_sel=sel, seed=3,
                              threads=16)
    assert got == want


def test_group_with_deletions(default_trace):
    rp = default_trace.replay(seed=9)
    keep = list(range(0, default_trace.num_nodes, 4))
    nodes = helpers.subset_nodes(rp, keep)
    evs, oev = helpers.delete_stream(default_trace, rp, 900, 0.3, seed=2)
    g = SH.ShardGroup(nodes, default_trace.typical(), 3)
    g.load_events(evs, len(evs))
    g.run()
    got = g.results()
    g.close()
    onodes = [helpers.oracle_nodes(default_trace, rp)[i] for i in keep]
    want, _, _ = O.run_events(onodes, helpers.oracle_typical(default_trace), oev, policy=O.POL_FGD,
                              gpu_sel=O.SEL_FGD, threads=16)
    assert got == want
    assert any(r[4] == ksim.DELETED and r[0] >= 0 for r in got)


def test_rccl_world1(default_trace):
    # the RCCL exchange (ncclAllGather, hipGraph-captured when the capture accepts it) at world 1
    rp = default_trace.replay(seed=42)
    n_ev = 2000
    arr, n = default_trace.typical()
    parts = SH.partition(rp.nodes, 1)
    e = ksim.Engine(default_trace.num_nodes, 1)
    e.set_shard(0, 1, 0, default_trace.num_nodes, ksim.shard_comm_id())
    e.set_nodes(0, parts[0][1])
    e.set_typical(0, arr, n)
    e.set_policy(0, "FGD")
    e.load_events(0, rp.events, n_ev)
    ms = e.run()
    got = SH.merge_results([e.results(0)], parts)
    e.close()
    assert got == unsharded(default_trace, rp.nodes, rp.events, n_ev, "FGD")
    print("sharded world 1 over RCCL: %d steps in %.1f ms (%.1f us/step)" % (n_ev, ms, ms * 1e3 / n_ev))
