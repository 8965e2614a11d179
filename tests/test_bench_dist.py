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
