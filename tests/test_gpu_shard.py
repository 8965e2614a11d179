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
    wgs = g.engines[0].last_run_wgs()
    g.close()
    assert wgs >= 1  # the FGD group ran on k_hmemo's sharded launch (K slices per shard)
    assert got == unsharded(default_trace, rp.nodes, rp.events, n_ev, "FGD")


@pytest.mark.parametrize("world", [2, 3])
def test_group_fgd_step_path_still_equal(default_trace, world, monkeypatch):
    # KSIM_VARIANT=shard_hmemo=0 keeps round 2's per-pod k_step + gather + commit path for an FGD group
    monkeypatch.setenv("KSIM_VARIANT", "shard_hmemo=0")
    rp = default_trace.replay(seed=43)
    n_ev = 600
    g = SH.ShardGroup(rp.nodes, default_trace.typical(), world)
    g.load_events(rp.events, n_ev)
    g.run()
    got = g.results()
    wgs = g.engines[0].last_run_wgs()
    g.close()
    assert wgs == 0
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
    kernels = g.engines[0].last_run_kernels()
    g.close()
    # FGD on k_hmemo slices, the other policies on k_replay slices (r06), each one launch for the group
    assert kernels == (["k_hmemo_group"] if name == "FGD" else ["k_replay_group"]), kernels
    onodes = helpers.oracle_subset(default_trace, rp, keep)
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
    onodes = helpers.oracle_subset(default_trace, rp, keep)
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


def _host_shard_engine(trace, nodes, n_ev, events, gather, policy="FGD"):
    arr, n = trace.typical()
    parts = SH.partition(nodes, 1)
    e = ksim.Engine(len(nodes), 1)
    e.set_shard(0, 1, 0, len(nodes))
    e.set_shard_exchange(gather)
    e.set_nodes(0, parts[0][1])
    e.set_typical(0, arr, n)
    e.set_policy(0, policy)
    e.load_events(0, events, n_ev)
    return e, parts


def test_host_exchange_world1(default_trace):
    # the host exchange (ksim_engine_set_shard_exchange) with the identity gather of a world of one
    rp = default_trace.replay(seed=42)
    n_ev = 800
    calls = []

    def gather(rec):
        calls.append(rec)
        return list(rec)
    e, parts = _host_shard_engine(default_trace, rp.nodes, n_ev, rp.events, gather)
    e.run()
    got = SH.merge_results([e.results(0)], parts)
    e.close()
    assert len(calls) == n_ev
    assert got == unsharded(default_trace, rp.nodes, rp.events, n_ev, "FGD")


@pytest.mark.parametrize("bad", ["raise", "size", "foreign"])
def test_host_exchange_bad_gather_fails(default_trace, bad):
    rp = default_trace.replay(seed=42)

    def gather(rec):
        if bad == "raise":
            raise RuntimeError("transport down")
        if bad == "size":
            return list(rec) + [0]
        return [rec[0] ^ 1] + list(rec[1:])  # not this shard's record at its rank
    e, _ = _host_shard_engine(default_trace, rp.nodes, 50, rp.events, gather)
    with pytest.raises(ksim.KsimError) as ei:
        e.run()
    e.close()
    assert ei.value.code == ksim.KSIM_ESTATE


def _device_rank_main(rank, world, port, n_ev, deletes, q, epoch0=None, n_runs=2):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if epoch0 is not None:
        os.environ["KSIM_TEST"] = "peer_epoch0=%s" % epoch0  # the run epoch starts just below its 24-bit wrap
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=7)
    nodes = helpers.subset_nodes(rp, list(range(1, t.num_nodes, 5)))
    events, n = rp.events, n_ev
    if deletes:
        events, _ = helpers.delete_stream(t, rp, n_ev, p_delete=0.2, seed=4)
        n = len(events)
    runs = []
    for _ in range(n_runs):  # several runs: each run's granules carry the next epoch over the last's
        runs.append(SH.run_distributed(nodes, t.typical(), events, n, dist, policy="FGD", seed=3, exchange="device"))
    q.put((rank, [r[0] for r in runs], runs[0][1]))
    dist.destroy_process_group()


@pytest.mark.timeout(150)
@pytest.mark.parametrize("deletes,epoch0,n_runs", [(False, None, 2), (True, None, 2), (False, "0xfffffe", 3)],
                         ids=["create", "delete", "epoch-wrap"])
def test_device_exchange_two_processes(default_trace, deletes, epoch0, n_runs):
    # two shard processes on the one GPU, each a persistent k_hmemo over its slices, exchanging per-pod
    # granules through each other's IPC-mapped buffers (the one-process-per-GPU mode's exchange; on a
    # node the peers' buffers sit on other GPUs, over xGMI).  epoch-wrap: three runs at epochs 0xffffff,
    # 1, 2 (the 24-bit run epoch wraps past 0), each bit-exact
    import multiprocessing as mp
    import socket
    n_ev = 600
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_device_rank_main, args=(r, 2, port, n_ev, deletes, q, epoch0, n_runs))
             for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=100) for _ in procs), key=lambda x: x[0])
    finally:
        for p in procs:
            if p.is_alive():
                p.join(20)
            if p.is_alive():
                p.kill()
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    rp = default_trace.replay(seed=7)
    keep = list(range(1, default_trace.num_nodes, 5))
    if deletes:
        events, oev = helpers.delete_stream(default_trace, rp, n_ev, p_delete=0.2, seed=4)
    else:
        oev = helpers.oracle_events(default_trace, rp, n_ev)
    want, _, _ = O.run_events(helpers.oracle_subset(default_trace, rp, keep), helpers.oracle_typical(default_trace),
                              oev, policy=O.POL_FGD, gpu_sel=O.SEL_FGD, seed=3, threads=16)
    for r in res:
        assert len(r[1]) == n_runs and all(run == want for run in r[1])
    print("device exchange world 2: %d events, rank times %.2f / %.2f ms" % (len(oev), res[0][2], res[1][2]))


def test_peer_handle_refusals(default_trace):
    # ksim_engine_set_shard_peers checks every peer's device before it maps anything: a handle naming a GPU
    # that is not visible here is KSIM_EPEER, a malformed one KSIM_EINVAL (include/ksim_engine.h)
    import struct
    rp = default_trace.replay(seed=7)
    nodes = helpers.subset_nodes(rp, list(range(0, default_trace.num_nodes, 8)))
    parts = SH.partition(nodes, 2)
    e = ksim.Engine(len(parts[0][2]), 1)
    try:
        e.set_shard(0, 2, parts[0][0], len(nodes), None)
        own = e.shard_peer_handle()
        assert len(own) == ksim.SHARD_HANDLE_BYTES and own[64:68] == b"KSPH"
        foreign = bytearray(own)
        foreign[68:80] = struct.pack("<III", 0xfff0, 0xfe, 0x1f)  # PCI fff0:fe:1f: no such GPU here
        with pytest.raises(ksim.KsimError) as ei:
            e.set_shard_peers([own, bytes(foreign)])
        assert ei.value.code == ksim.KSIM_EPEER
        bad = bytearray(own)
        bad[64:68] = b"XXXX"
        with pytest.raises(ksim.KsimError) as ei:
            e.set_shard_peers([own, bytes(bad)])
        assert ei.value.code == ksim.KSIM_EINVAL
    finally:
        e.close()


def _host_rank_main(rank, world, port, policy, n_ev, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=7)
    nodes = helpers.subset_nodes(rp, list(range(1, t.num_nodes, 5)))
    merged, ms = SH.run_distributed(nodes, t.typical(), rp.events, n_ev, dist, policy=policy, seed=3,
                                    exchange="host")
    q.put((rank, merged, ms))
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,pol,sel", [POLICIES[0], POLICIES[1]], ids=["FGD", "BestFit"])
def test_host_exchange_two_processes(default_trace, name, pol, sel):
    # two shard processes on the one GPU, their per-step records exchanged over gloo: the shard
    # kernels and the commit of the multi-process mode with a real cross-process exchange (RCCL
    # refuses two ranks on one device, so the ncclAllGather itself stays world-1 here)
    # stdlib multiprocessing: the ranks import torch.distributed for the gloo gather; ksim binds them to
    # torch's HIP runtime (ksim.hip_runtime_path), one runtime per process
    import multiprocessing as mp
    import socket
    n_ev = 600
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_host_rank_main, args=(r, 2, port, name, n_ev, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=200) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    rp = default_trace.replay(seed=7)
    keep = list(range(1, default_trace.num_nodes, 5))
    onodes = helpers.oracle_subset(default_trace, rp, keep)
    want, _, _ = O.run_events(onodes, helpers.oracle_typical(default_trace),
                              helpers.oracle_events(default_trace, rp, n_ev), policy=pol, gpu_sel=sel, seed=3,
                              threads=16)
    assert res[0][1] == want and res[1][1] == want
    print("host exchange world 2 (%s): %d steps, rank times %.1f / %.1f ms" % (name, n_ev, res[0][2], res[1][2]))
