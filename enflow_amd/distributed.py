"""One-process-per-GPU helpers (torch.distributed; backend "nccl" is RCCL on ROCm).

The flow shards naturally: molecules are independent, so forward / inverse
run with no collective at all (each rank owns a contiguous molecule range).
Training adds one gradient all-reduce per step; gradients are flattened into
a few large buckets (xGMI is point-to-point: fewer, larger ring all-reduces).
"""
import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 64 << 20


def shard_range(num_units, rank, world):
    """Contiguous, balanced [start, end) share of `num_units` for `rank`."""
    base, rem = divmod(num_units, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def max_over_ranks(value, device=None):
    """Max of a host float over all ranks (the bench's timing rule)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_gradients(params, bucket_bytes=DEFAULT_BUCKET_BYTES, average=True):
    """Sum (or average) .grad of `params` over ranks with bucketed flat all-reduces."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size()
    if world == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    bucket, size = [], 0
    for g in grads + [None]:
        if g is not None:
            bucket.append(g)
            size += g.numel() * g.element_size()
        if bucket and (g is None or size >= bucket_bytes):
            flat = torch.cat([b.reshape(-1) for b in bucket])
            dist.all_reduce(flat)
            if average:
                flat /= world
            off = 0
            for b in bucket:
                n = b.numel()
                b.copy_(flat[off:off + n].view_as(b))
                off += n
            bucket, size = [], 0
