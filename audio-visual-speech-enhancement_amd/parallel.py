"""Clip sharding across the GPUs of one node (one process per GPU) + the final RCCL gather.

The reference has no parallelism (`--gpus` is parsed and never read,
speech_enhancer.py:283, :289).  Clips (200-ms segments) are independent, so the batch is split into
contiguous per-rank blocks with no data-path collective; the only exchanges are a one-time weight
broadcast and one all-gather of the [n, 80, 20] outputs.  With backend "nccl" this is RCCL over
xGMI; the same code runs on "gloo" for CPU tests.
"""
import torch
import torch.distributed as dist


def shard_bounds(n, world, rank):
    """Contiguous block of clips [start, stop) owned by `rank` (sizes differ by at most one)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard(x, world=None, rank=None):
    world = dist.get_world_size() if world is None else world
    rank = dist.get_rank() if rank is None else rank
    a, b = shard_bounds(x.shape[0], world, rank)
    return x[a:b]


def broadcast_(t, src=0):
    """One-time replication (e.g. the weight blob) from `src`."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src)
    return t


def gather_clips(local, n_total):
    """All-gather every rank's contiguous block back into [n_total, ...] (rank order = clip order).

    Blocks are padded to ceil(n_total / world) so one all_gather_into_tensor (RCCL) moves them."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    per = -(-n_total // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    if dist.get_backend() == "nccl":
        out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, pad)
        parts = list(out.split(per))
    else:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
    return torch.cat([p[: (lambda ab: ab[1] - ab[0])(shard_bounds(n_total, world, r))] for r, p in enumerate(parts)])


def sharded_predict(network, mixed, video, video_normalizer=None):
    """Every rank holds the full batch (or the same seeded inputs); each computes its block on its
    own GPU and the blocks are all-gathered, so every rank returns the full [n, 80, 20]."""
    n = mixed.shape[0]
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    a, b = shard_bounds(n, world, rank)
    local = network.predict_device(mixed[a:b], video[a:b], video_normalizer)
    return gather_clips(local, n)
