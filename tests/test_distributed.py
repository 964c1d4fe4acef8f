"""world_size-2 gloo tests (CPU) of the multi-process path: molecule sharding,
max-over-ranks timing and the bucketed gradient all-reduce."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from enflow_amd.distributed import shard_range, max_over_ranks, allreduce_gradients


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        out["shard"] = shard_range(1027, rank, world)
        out["max"] = max_over_ranks(1.5 + rank)
        torch.manual_seed(rank)
        params = [torch.nn.Parameter(torch.zeros(s)) for s in ((3, 4), (7,), (128, 5))]
        for p in params:
            p.grad = torch.randn_like(p)
        local = [p.grad.clone() for p in params]
        allreduce_gradients(params, bucket_bytes=64)   # tiny buckets: exercise bucketing
        # plain lists: a tensor put on a multiprocessing queue is shared through
        # the sender's file descriptors, which vanish if this process exits first
        out["grads"] = [p.grad.tolist() for p in params]
        out["local"] = [t.tolist() for t in local]
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s0, s1 = res[0]["shard"], res[1]["shard"]
    assert s0[0] == 0 and s0[1] == s1[0] and s1[1] == 1027 and abs((s0[1] - s0[0]) - (s1[1] - s1[0])) <= 1
    assert res[0]["max"] == res[1]["max"] == 2.5
    T = torch.tensor
    for g0, g1, l0, l1 in zip(res[0]["grads"], res[1]["grads"], res[0]["local"], res[1]["local"]):
        g0, g1, l0, l1 = T(g0), T(g1), T(l0), T(l1)
        torch.testing.assert_close(g0, (l0 + l1) / 2)
        torch.testing.assert_close(g1, (l0 + l1) / 2)


@pytest.mark.parametrize("n,world", [(1024, 8), (10, 3), (3, 4), (0, 2)])
def test_shard_range_partitions(n, world):
    ranges = [shard_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
