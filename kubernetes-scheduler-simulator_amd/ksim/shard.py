"""Node-sharded single cluster (C5 across GPUs) -- host side.

The cluster's nodes are split into `world` contiguous ranges of name rank (the selectHost key,
generic_scheduler.go:187-212), one engine per range.  Every shard sees every event; per pod the
shards exchange a 32-byte record and only the owner of the winning node binds
(ksim_engine_set_shard).  This module builds the shards from a global node list and merges the
per-shard results back into global results (node = the input index, as an unsharded engine reports).
"""
import ctypes as C

import ksim


def partition(nodes, world):
    """Split a global ksim.Node array into `world` shards by name rank.
    Returns [(offset, local ksim.Node array ordered by rank, [global input index of each local node])]."""
    n = len(nodes)
    by_rank = sorted(range(n), key=lambda i: nodes[i].name_rank)
    assert [nodes[i].name_rank for i in by_rank] == list(range(n)), "name ranks must be 0..N-1"
    out = []
    for k in range(world):
        lo, hi = k * n // world, (k + 1) * n // world
        arr = (ksim.Node * max(1, hi - lo))()
        for j, i in enumerate(by_rank[lo:hi]):
            C.memmove(C.byref(arr[j]), C.byref(nodes[i]), C.sizeof(ksim.Node))
        out.append((lo, arr, by_rank[lo:hi]))
    return out


def merge_results(per_shard, parts):
    """Global results from the shards' results: per step, the record of the shard that owns the
    reported node (global rank) is authoritative; node ranks become input indices."""
    index_of_rank = {}
    owner_of_rank = {}
    for k, (off, _, idx) in enumerate(parts):
        for j, i in enumerate(idx):
            index_of_rank[off + j] = i
            owner_of_rank[off + j] = k
    out = []
    for s in range(len(per_shard[0])):
        r = per_shard[0][s]
        if r[0] >= 0:
            r = per_shard[owner_of_rank[r[0]]][s]
        node = index_of_rank[r[0]] if r[0] >= 0 else -1
        out.append((node,) + tuple(r[1:]))
    return out


class ShardGroup:
    """`world` shards of one cluster on one device, run in lockstep (ksim_shard_group_run)."""

    def __init__(self, nodes, typical, world, policy="FGD", seed=0, device=0, report=False):
        arr, n = typical
        self.parts = partition(nodes, world)
        self.engines = []
        for k, (off, local, idx) in enumerate(self.parts):
            e = ksim.Engine(len(idx), 1, device=device)
            e.set_shard(k, world, off, len(nodes))
            e.set_nodes(0, local)
            e.set_typical(0, arr, n)
            e.set_policy(0, policy, seed=seed)
            if report:
                e.set_report(True)
            self.engines.append(e)

    def load_events(self, events, n):
        for e in self.engines:
            e.load_events(0, events, n)

    def run(self):
        return ksim.shard_group_run(self.engines)

    def results(self):
        return merge_results([e.results(0) for e in self.engines], self.parts)

    def close(self):
        for e in self.engines:
            e.close()


def host_gather(dist, group=None):
    """A ksim_shard_exchange_fn body over torch.distributed (any backend with CPU tensors, e.g.
    gloo): all-gather of the 4-word shard record, returned flat in rank order."""
    import torch
    world = dist.get_world_size(group)

    def signed(v):
        return v - (1 << 64) if v >= 1 << 63 else v

    def gather(record):
        t = torch.tensor([signed(v) for v in record], dtype=torch.int64)
        out = [torch.empty(4, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return [int(v) & 0xFFFFFFFFFFFFFFFF for o in out for v in o.tolist()]
    return gather


def run_distributed(nodes, typical, events, n, dist, policy="FGD", seed=0, device=0, engine_cls=None,
                    exchange="rccl"):
    """One shard per process (torchrun; backend nccl = RCCL for the launcher's own collectives):
    rank 0 makes the RCCL id of the shards' exchange, every rank builds its shard engine on
    `device`, replays the events, and the per-shard results are gathered and merged on every rank.
    exchange="host": no RCCL communicator; every pod step's record goes through `dist` (host_gather),
    e.g. shards sharing one GPU, or hosts without a common RCCL fabric.
    exchange="device" (FGD): each shard's persistent k_hmemo stores its per-step slice maxima straight into
    every peer's IPC-mapped exchange buffer (ksim_engine_set_shard_peers); `dist` only carries the handles.
    Returns (merged results, device ms of this rank's run)."""
    engine_cls = engine_cls or ksim.Engine
    rank, world = dist.get_rank(), dist.get_world_size()
    parts = partition(nodes, world)
    off, local, idx = parts[rank]
    if exchange == "rccl":
        box = [shard_comm_id_for(engine_cls) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
    elif exchange in ("host", "device"):
        box = [None]
    else:
        raise ValueError("exchange must be 'rccl', 'host' or 'device'")
    e = engine_cls(len(idx), 1, device=device)
    e.set_shard(rank, world, off, len(nodes), box[0])
    if exchange == "host":
        e.set_shard_exchange(host_gather(dist))
    if exchange == "device":  # FGD: the shards' k_hmemo slices exchange granules through IPC-mapped buffers
        handles = [None] * world
        dist.all_gather_object(handles, e.shard_peer_handle())
        e.set_shard_peers(handles)
    e.set_nodes(0, local)
    arr, nt = typical
    e.set_typical(0, arr, nt)
    e.set_policy(0, policy, seed=seed)
    e.load_events(0, events, n)
    ms = e.run()
    mine = e.results(0)
    e.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    return merge_results(gathered, parts), ms


def shard_comm_id_for(engine_cls):
    f = getattr(engine_cls, "comm_id", None)
    return f() if f is not None else ksim.shard_comm_id()
