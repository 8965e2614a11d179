"""The node-sharded driver's host path on CPU: partition by name rank, result
merge, and the world-size-2 gloo protocol of ksim.shard.run_distributed (comm-id broadcast,
per-shard results gathered and merged).  The shard engine is replaced by a stand-in that derives
each shard's view from the oracle's unsharded decisions, so the merge must give them back."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-scheduler-simulator_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import ksim  # noqa: E402
import ksim.shard as SH  # noqa: E402


def _nodes(n, ranks):
    arr = (ksim.Node * n)()
    for i in range(n):
        arr[i].name_rank = ranks[i]
        arr[i].gpu_count = 1 + i % 8
    return arr


def test_partition_contiguous_ranks():
    ranks = [5, 0, 3, 1, 4, 2, 6]
    parts = SH.partition(_nodes(7, ranks), 3)
    assert [p[0] for p in parts] == [0, 2, 4]
    for off, local, idx in parts:
        for j, i in enumerate(idx):
            assert local[j].name_rank == off + j and ranks[i] == off + j


def _views(full, parts, world):
    """Each shard's result stream as the device writes it: the owner of the winning node has the
    real record, the others the winner's global rank with gpu_mask 0 (ksim_engine.h)."""
    rank_of = {}
    owner = {}
    for k, (off, _, idx) in enumerate(parts):
        for j, i in enumerate(idx):
            rank_of[i] = off + j
            owner[off + j] = k
    views = []
    for k in range(world):
        v = []
        for (node, mask, score, nf, st) in full:
            if node < 0:
                v.append((node, mask, score, nf, st))
            else:
                r = rank_of[node]
                v.append((r, mask, score, nf, st) if owner[r] == k else (r, 0, score, nf, 0))
        views.append(v)
    return views


def test_merge_results_owner_wins():
    parts = SH.partition(_nodes(6, [3, 1, 0, 5, 2, 4]), 2)
    full = [(0, 1, 100000, 6, 0), (-1, 0, 0, 0, 1), (3, 4, 99000, 5, 0), (5, 2, 0, 1, 0)]
    assert SH.merge_results(_views(full, parts, 2), parts) == full


class OracleShard:
    """Stand-in shard engine: its results are its view of the oracle's unsharded decisions."""
    full = None
    all_nodes = None

    def __init__(self, n, r, device=0):
        self.n = n

    @staticmethod
    def comm_id():
        return b"\x07" * ksim.SHARD_ID_BYTES

    def set_shard(self, rank, world, off, n_global, comm_id):
        assert comm_id == b"\x07" * ksim.SHARD_ID_BYTES and n_global == len(OracleShard.all_nodes)
        self.rank, self.world = rank, world

    def set_nodes(self, r, nodes):
        self.local = nodes

    def set_typical(self, *a):
        pass

    def set_policy(self, *a, **k):
        pass

    def load_events(self, *a):
        pass

    def run(self):
        return 0.0

    def results(self, r):
        parts = SH.partition(OracleShard.all_nodes, self.world)
        return _views(OracleShard.full, parts, self.world)[self.rank]

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    import helpers
    import pyoracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = ksim.Trace.openb("default")
    rp = t.replay(seed=42)
    keep = list(range(0, t.num_nodes, 10))
    nodes = helpers.subset_nodes(rp, keep)
    onodes = helpers.oracle_subset(t, rp, keep)
    full, _, _ = O.run_events(onodes, helpers.oracle_typical(t), helpers.oracle_events(t, rp, 300), threads=1)
    OracleShard.full, OracleShard.all_nodes = full, nodes
    merged, _ = SH.run_distributed(nodes, t.typical(), rp.events, 300, dist, engine_cls=OracleShard)
    q.put((rank, merged == full, sum(1 for r in full if r[0] >= 0)))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_gloo_world2_sharded_protocol():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True, True] and res[0][2] > 100


def _gather_main(rank, world, port, q):
    import ctypes as C
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fn = ksim.exchange_cfunc(SH.host_gather(dist), world)
    send = (C.c_uint64 * 4)(0xFFFFFFFFFFFFFFFF - rank, rank, 1 << 63 | rank, 12345 + rank)
    recv = (C.c_uint64 * (4 * world))()
    rc = fn(send, recv, None)  # called through the C function pointer, as the engine calls it
    bad = ksim.exchange_cfunc(lambda rec: rec, world)(send, recv, None)  # a wrong-sized gather
    q.put((rank, rc, bad, list(recv)))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_host_gather():
    # the host-exchange transport of ksim.shard.run_distributed(exchange="host"): the 4-word u64
    # records of both ranks, high bit included, in rank order on every rank
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    want = [0xFFFFFFFFFFFFFFFF, 0, 1 << 63, 12345, 0xFFFFFFFFFFFFFFFE, 1, (1 << 63) | 1, 12346]
    for rank, rc, bad, recv in res:
        assert rc == 0 and bad == 1 and recv == want
