"""The real HIP forward in more than one process: two ranks on the one GPU of the box, gloo for the
collectives (RCCL refuses two ranks on one device, profiles/r05f_rccl_probe.log), outputs staged through host memory by
parallel.gather_clips.  Each rank runs libavse's float32_split forward on its contiguous block with real DeviceWeights:

  * parallel.sharded_predict  (network.py:208-212 sharded by clips)       N = 37 and 1080 clips
  * parallel.sharded_enhance  (pipeline.Enhancer sharded by utterances)   5 three-second utterances (3 / 2 per rank)
  * `speech_enhancer.py predict -g 2` (speech_enhancer.py:283, :289)      AVSE_DIST_BACKEND=gloo, 4 samples

and the gathered results / written wav files must be bitwise equal to the single-process run (the fp32-accurate forward
is batch-invariant, tests/test_gpu_split.py::test_fp32_forward_is_batch_invariant), every sample written once."""
import glob
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPLIT = "float32_split"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(n, seed):
    from conftest import synth_video
    rng = np.random.default_rng(seed)
    mel = rng.normal(-40, 15, (n, 80, 20)).astype(np.float32)
    video = synth_video(rng, n)
    return mel, video, video.mean(axis=(0, 3)).astype(np.float32), video.std(axis=(0, 3)).astype(np.float32)


def _utterances(u, seed):
    from conftest import synth_audio
    rng = np.random.default_rng(seed)
    sig = synth_audio(rng, u, 48000)
    video = rng.integers(0, 256, (u, 15, 128, 128, 5)).astype(np.float32)
    return sig, video, video.reshape(-1, 128, 128, 5).mean(axis=(0, 3)).astype(np.float32), \
        video.reshape(-1, 128, 128, 5).std(axis=(0, 3)).astype(np.float32)


def _model():
    from avse_amd.model import KerasModel
    return KerasModel.init(seed=21, randomize=True)


class _Norm:
    """VideoNormalizer stand-in with fixed device statistics (data_processor.VideoNormalizer.device_stats)."""

    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def device_stats(self, dev):
        from avse_amd import ops
        return ops.to_device(self.mean, dev), ops.to_device(self.std, dev)


def _single(n_list, u):
    """The single-process results the sharded runs must reproduce."""
    from avse_amd import ops
    from avse_amd.network import SpeechEnhancementNetwork
    from avse_amd.pipeline import Enhancer
    net = SpeechEnhancementNetwork(_model(), SPLIT)
    preds = {}
    for n in n_list:
        mel, video, m, s = _inputs(n, n)
        preds[n] = net.predict_device(mel, video, _Norm(m, s)).cpu().numpy()
    sig, vid, m, s = _utterances(u, 7)
    enh = Enhancer(net.device_weights())(ops.to_device(sig), ops.to_device(vid), ops.to_device(m), ops.to_device(s))
    return preds, enh.cpu().numpy()


def _worker(rank, world, port, n_list, u, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import avse_pkg
    avse_pkg.load()
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from avse_amd import ops, parallel
        from avse_amd.network import SpeechEnhancementNetwork
        from avse_amd.pipeline import Enhancer
        net = SpeechEnhancementNetwork(_model(), SPLIT)
        res = {"rank": rank, "pred": {}, "rows": {}}
        for n in n_list:
            mel, video, m, s = _inputs(n, n)
            a, b = parallel.shard_bounds(n, world, rank)
            # data loaded per rank (n_total given): only this rank's block ever reaches its device
            full = parallel.sharded_predict(net, mel[a:b], video[a:b], _Norm(m, s), n_total=n)
            res["pred"][n] = full.cpu().numpy()
            res["rows"][n] = b - a
        sig, vid, m, s = _utterances(u, 7)
        a, b = parallel.shard_bounds(u, world, rank)
        enh = Enhancer(net.device_weights())
        out = parallel.sharded_enhance(enh, ops.to_device(sig[a:b]), ops.to_device(vid[a:b]), ops.to_device(m),
                                       ops.to_device(s), n_total=u)
        res["enh"] = out.cpu().numpy()
        res["range_bits"] = enh.range_bits
        q.put(res)
    except Exception as e:  # noqa: BLE001 — reported to the parent
        import traceback
        q.put({"rank": rank, "error": repr(e) + "\n" + traceback.format_exc()})
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_sharded_predict_and_enhance(gpu):
    import torch.multiprocessing as mp
    n_list, u, world = (37, 1080), 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_list, u, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    errs = [r["error"] for r in res if "error" in r]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    preds, enh = _single(n_list, u)
    for n in n_list:
        assert [r["rows"][n] for r in res] == [-(-n // 2), n // 2]          # contiguous blocks, the last shorter
        for r in res:
            assert r["pred"][n].shape == preds[n].shape
            diff = float(np.abs(r["pred"][n] - preds[n]).max())
            print(f"N={n} rank {r['rank']}: gathered forward vs one process max |diff| {diff:.3g}")
            assert np.array_equal(r["pred"][n], preds[n]), (n, r["rank"], diff)
    for r in res:
        assert r["range_bits"] == 0
        assert r["enh"].shape == enh.shape == (u, 160 * (15 * 20 - 1))
        assert np.array_equal(r["enh"], enh), float(np.abs(r["enh"] - enh).max())


def test_cli_predict_two_ranks_gloo_on_one_gpu(gpu, tmp_path):
    """`predict -g 2` (torch.distributed.run, 2 ranks, AVSE_DIST_BACKEND=gloo on the box's one GPU) against `predict`
    in one process: the same losses in sample order and the same wav files bit for bit, each sample written once."""
    from test_gpu_cli import make_dataset, run
    tmp = str(tmp_path)
    ds, noise = make_dataset(tmp, n_noise=4)
    base = os.path.join(tmp, "base")
    os.makedirs(base)
    assert "preprocessed 4 samples" in run(["-bd", base, "preprocess", "-dn", "d", "-ds", ds, "-n", noise], tmp)
    run(["-bd", base, "train", "-mn", "m", "-tdn", "d", "-vdn", "d", "--init-only"], tmp)
    results = {}
    for mode in ("one", "two"):
        args = [sys.executable, os.path.join(ROOT, "speech_enhancer.py"), "-bd", base, "predict", "-mn", "m", "-dn", "d"]
        env = dict(os.environ)
        if mode == "two":
            args += ["-g", "2"]
            env["AVSE_DIST_BACKEND"] = "gloo"
        r = subprocess.run(args, cwd=tmp, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        losses = [ln for ln in r.stdout.splitlines() if ln.startswith("loss:")]
        assert len(losses) == 4, r.stdout + r.stderr
        run_dir = os.path.join(base, "out", "m", "d")
        wavs = sorted(glob.glob(os.path.join(run_dir, "*", "*", "*", "enhanced.wav")))
        assert len(wavs) == 4 and len(os.listdir(run_dir)) == 1      # one run directory for both ranks
        results[mode] = (losses, {os.path.join(*w.split(os.sep)[-3:]): open(w, "rb").read() for w in wavs})
        shutil.move(run_dir, run_dir + "_" + mode)
    assert results["one"][0] == results["two"][0]
    assert results["one"][1].keys() == results["two"][1].keys()
    for k in results["one"][1]:
        assert results["one"][1][k] == results["two"][1][k], k
