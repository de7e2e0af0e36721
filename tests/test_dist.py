"""Multi-process (gloo, world_size 2 and 3) tests of the clip sharding + final gather used on the
GPU path (RCCL there).  The per-rank "forward" is a deterministic CPU stand-in; what is tested is
that every clip is computed exactly once and comes back in order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import avse_pkg
    avse_pkg.load()
    from avse_amd import parallel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        x = torch.randn(n, 80, 20, generator=g)
        a, b = parallel.shard_bounds(n, world, rank)
        local = torch.tanh(x[a:b]) * 3 + rank * 0          # stand-in per-clip computation
        full = parallel.gather_clips(local, n)
        w = torch.arange(10, dtype=torch.float32) if rank == 0 else torch.zeros(10)
        parallel.broadcast_(w, 0)
        q.put((rank, bool(torch.equal(full, torch.tanh(x) * 3)), bool(torch.equal(w, torch.arange(10.0)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 512), (2, 7), (3, 10), (2, 1)])
def test_gather_reassembles_every_clip_in_order(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and bok for _, ok, bok in res), res


class StandInNetwork:
    """Duck-typed SpeechEnhancementNetwork: predict_device is a per-clip CPU function (gloo, no GPU)."""

    def __init__(self):
        self.seen = 0

    def predict_device(self, mixed, video, video_normalizer=None):
        self.seen += mixed.shape[0]
        return torch.tanh(mixed) + video.mean(dim=(1, 2, 3))[:, None, None]


def stand_in_enhancer(signals, video, vmean=None, vstd=None):
    """Duck-typed pipeline.Enhancer: per-utterance output of a different length than the input."""
    return signals[:, ::2] * 0.5 + video.sum(dim=(1, 2, 3, 4))[:, None]


def _predict_worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import avse_pkg
    avse_pkg.load()
    from avse_amd import parallel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1)
        mixed = torch.randn(n, 80, 20, generator=g)
        video = torch.randn(n, 8, 8, 5, generator=g)
        ref = StandInNetwork().predict_device(mixed, video)
        net = StandInNetwork()
        full = parallel.sharded_predict(net, mixed, video)                 # every rank holds the whole batch
        a, b = parallel.shard_bounds(n, world, rank)
        net2 = StandInNetwork()
        full2 = parallel.sharded_predict(net2, mixed[a:b], video[a:b], n_total=n)   # data loaded per rank
        # utterance sharding of the end-to-end path: 3 slices per utterance, 600-sample signals
        sig = torch.randn(n, 600, generator=g)
        vid = torch.randn(n, 3, 4, 4, 5, generator=g)
        enh = parallel.sharded_enhance(stand_in_enhancer, sig[a:b], vid[a:b], n_total=n)
        q.put((rank, bool(torch.equal(full, ref)), bool(torch.equal(full2, ref)), net.seen == b - a,
               net2.seen == b - a, bool(torch.equal(enh, stand_in_enhancer(sig, vid)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (3, 11), (2, 1)])
def test_sharded_predict_and_enhance_uneven_last_shard(world, n):
    """parallel.sharded_predict / sharded_enhance with duck-typed stand-ins: each rank computes exactly its
    contiguous block (the last one shorter), and every rank gets the full result in order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_predict_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(all(r[1:]) for r in res), res


def test_shard_bounds_cover_exactly_once():
    import avse_pkg
    avse_pkg.load()
    from avse_amd.parallel import shard_bounds
    for n in range(0, 40):
        for w in range(1, 9):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
