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


def _cli_worker(rank, world, port, n, fail_at, outdir, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import avse_pkg
    avse_pkg.load()
    import numpy as np
    from avse_amd import speech_enhancer as se
    from avse_amd.audio_io import AudioSignal
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        samples = []
        for i in range(n):
            S = 15 if i % 3 else 10          # two shape groups
            samples.append(se.Sample("spk%d" % (i % 2), "v%d.npy" % i, "s%d.wav" % i, "n%d.wav" % i,
                                     rng.normal(size=(S, 4, 4, 5)).astype(np.float32),
                                     rng.normal(size=(S, 80, 20)).astype(np.float32),
                                     rng.normal(size=(S, 80, 20)).astype(np.float32), None,
                                     AudioSignal(rng.normal(size=3200 * S).astype(np.float32), 16000), 25.0))
        calls = []

        def stand_in(group):                 # duck-typed BatchPredictor: per-sample loss and "signal"
            calls.append(len(group))
            if any(g.video_file_path == "v%d.npy" % fail_at for g in group):
                raise RuntimeError("stand-in failure")
            return [(float(np.mean((g.mixed_spectrograms - g.speech_spectrograms) ** 2)),
                     AudioSignal(g.mixed_signal.get_data()[::2] * 0.5, 16000)) for g in group]

        def write(run_dir, smp, signal):
            with open(os.path.join(run_dir, os.path.basename(smp.video_file_path) + ".%d" % rank), "wb") as fh:
                fh.write(np.asarray(signal.get_data(), np.float32).tobytes())

        losses = se.predict_samples(samples, stand_in, outdir, world, rank, write=write,
                                    fallback=lambda smp: stand_in([smp])[0] if smp.video_file_path != "v%d.npy" % fail_at
                                    else (_ for _ in ()).throw(RuntimeError("stand-in failure")))
        expect = {i: float(np.mean((s.mixed_spectrograms - s.speech_spectrograms) ** 2)) for i, s in enumerate(samples)}
        expect[fail_at] = None
        q.put((rank, losses == expect if rank == 0 else True, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (3, 11)])
def test_sharded_cli_predict_writes_every_sample_once(world, n, tmp_path):
    """speech_enhancer.predict_samples under `predict -g N` (gloo here, RCCL on the GPUs): each rank batches its
    contiguous block of samples per shape group, writes the outputs of the samples it owns, a failing sample is
    skipped alone (its group retried sample by sample), and rank 0 gathers every loss in sample order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    fail_at = 3
    procs = [ctx.Process(target=_cli_worker, args=(r, world, port, n, fail_at, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    written = sorted(os.listdir(tmp_path))
    names = [w.rsplit(".", 1)[0] for w in written]
    assert sorted(names) == sorted("v%d.npy" % i for i in range(n) if i != fail_at)   # each once, failure skipped
    assert any(c > 1 for _, _, calls in res for c in calls)                           # groups ran batched
