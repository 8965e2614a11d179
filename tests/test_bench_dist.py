"""The N>1 bench path on CPU: world_size-2 gloo ranks exercise bench.py's seed
sharding and job reduction (max time over ranks, summed events) exactly as the
nccl ranks do on the GPU node -- replicas only, no data-path collective."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    seeds = bench.seeds_for_rank(rank, 10)
    dt, ev = bench.reduce_job(1.0 + rank, 1000 * (rank + 1), dist, "cpu")
    out.put((rank, seeds, dt, ev))
    dist.destroy_process_group()


def test_seeds_disjoint_and_c2_on_rank0():
    import bench
    s0, s1 = bench.seeds_for_rank(0, 10), bench.seeds_for_rank(1, 10)
    assert s0 == list(range(42, 52))  # C2's seeds on rank 0
    assert not set(s0) & set(s1)


def test_reduce_job_single_process():
    import bench
    assert bench.reduce_job(2.5, 77) == (2.5, 77)


@pytest.mark.timeout(120)
def test_gloo_world2_job_reduction():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (r0, s0, dt0, ev0), (r1, s1, dt1, ev1) = res
    assert dt0 == dt1 == 2.0          # max over ranks
    assert ev0 == ev1 == 3000         # summed events
    assert s0 == list(range(42, 52)) and s1 == list(range(52, 62))


class _StubEngine:
    """Stands in for ksim.Engine (no GPU here): records what bench._sharded_engine hands the engine."""
    calls = []

    def __init__(self, n_nodes, n_replicas, device=0, **kw):
        self.n, self.R, self.rank = n_nodes, n_replicas, None
        _StubEngine.calls.append(("create", n_nodes, n_replicas))

    def set_shard(self, rank, world, off, n_global, comm_id):
        self.rank = rank
        _StubEngine.calls.append(("set_shard", rank, world, off, n_global, comm_id))

    def shard_peer_handle(self):
        import ksim
        return (b"IPC%d" % self.rank).ljust(64, b"\0") + b"KSPH" + bytes(ksim.SHARD_HANDLE_BYTES - 68)

    def set_shard_peers(self, handles):
        _StubEngine.calls.append(("peers", list(handles)))

    def set_nodes(self, r, nodes):
        _StubEngine.calls.append(("nodes", r, [nodes[i].name_rank for i in range(len(nodes))]))

    def set_typical(self, r, arr, n):
        pass

    def set_policy(self, r, pol):
        _StubEngine.calls.append(("policy", r, pol))

    def load_events(self, r, events, n):
        _StubEngine.calls.append(("events", r, n))


def _sharded_rank_main(rank, world, port, out):
    # bench.py --config c5 --sharded's engine set-up (bench._sharded_engine) on a real gloo world, with the
    # engine stubbed: the IPC handles go round in rank order, every shard sees the same list
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import ksim
    bench.ksim.Engine = _StubEngine
    t = ksim.Trace.openb("default")
    eng = bench._sharded_engine(0, rank, world, t, dist)
    out.put((rank, _StubEngine.calls, eng.total_events, t.num_nodes))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_gloo_world2_sharded_handle_exchange():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    offs, sizes = [], []
    for rank, calls, n_ev, n_global in res:
        kinds = [c[0] for c in calls]
        # the order the engine needs: shard before peers before nodes (include/ksim_engine.h)
        assert kinds.index("set_shard") < kinds.index("peers") < kinds.index("nodes")
        _, r, world, off, ng, comm = calls[kinds.index("set_shard")]
        assert (r, world, ng, comm) == (rank, 2, n_global, None)  # device exchange: no RCCL comm id
        peers = calls[kinds.index("peers")][1]
        assert [h[:4] for h in peers] == [b"IPC0", b"IPC1"]        # rank order, this shard's own at its rank
        ranks = calls[kinds.index("nodes")][2]
        assert ranks == list(range(off, off + len(ranks)))           # local node i has global name rank off + i
        assert calls[kinds.index("events")][2] == n_ev > 0
        offs.append(off)
        sizes.append(len(ranks))
    assert offs[0] == 0 and offs[1] == sizes[0] and sum(sizes) == res[0][3]  # the shards tile the cluster
