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
        # gloo (CPU tests; several ranks sharing one GPU, where RCCL refuses duplicate devices): stage through host
        # memory, then back onto the rank's device
        host = pad.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host)
        parts = [p.to(local.device) for p in parts]
    return torch.cat([p[: (lambda ab: ab[1] - ab[0])(shard_bounds(n_total, world, r))] for r, p in enumerate(parts)])


def _local_block(x, n_total):
    """(this rank's rows, the global row count): x is either the full batch (n_total None) or already this
    rank's contiguous block of an n_total-row batch (data loaded per rank)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if n_total is None:
        a, b = shard_bounds(x.shape[0], world, rank)
        return x[a:b], x.shape[0]
    a, b = shard_bounds(n_total, world, rank)
    if x.shape[0] != b - a:
        raise ValueError(f"rank {rank} holds {x.shape[0]} rows, its block of {n_total} is {b - a}")
    return x, n_total


def sharded_predict(network, mixed, video, video_normalizer=None, n_total=None):
    """Clip-sharded SpeechEnhancementNetwork.predict (network.py:208-212): each rank runs the forward on its
    contiguous block of clips on its own GPU and the blocks are all-gathered, so every rank returns the full
    [n_total, 80, 20] in clip order.  mixed / video: the full batch (n_total None) or this rank's block."""
    local_mixed, n = _local_block(mixed, n_total)
    local_video, _ = _local_block(video, n_total)
    local = network.predict_device(local_mixed, local_video, video_normalizer)
    return gather_clips(local, n)


def sharded_enhance(enhancer, signals, video, vmean=None, vstd=None, n_total=None):
    """Utterance-sharded end-to-end enhancement (pipeline.Enhancer, BASELINE configs[4]): the STFT's top_db
    is per utterance, so whole utterances are the unit; every rank enhances its block and the enhanced
    signals are all-gathered in utterance order.  signals / video: all utterances or this rank's block."""
    local_sig, n = _local_block(signals, n_total)
    local_vid, _ = _local_block(video, n_total)
    return gather_clips(enhancer(local_sig, local_vid, vmean, vstd), n)
