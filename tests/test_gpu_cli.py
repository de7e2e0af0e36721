"""Config 1 (BASELINE.json configs[0]): preprocess -> train --init-only -> predict through the CLI on a
synthetic 2-speaker x 2-clip dataset with one noise file (list_data zips to min(4, 1) = 1 sample,
speech_enhancer.py:208)."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def make_dataset(tmp, n_noise=1):
    from scipy.io import wavfile
    rng = np.random.default_rng(0)
    ds = os.path.join(tmp, "dataset")
    for spk in ("s1", "s2"):
        os.makedirs(os.path.join(ds, spk, "audio"))
        os.makedirs(os.path.join(ds, spk, "video"))
        for clip in ("a", "b"):
            t = np.arange(48000) / 16000
            speech = (3000 * np.sin(2 * np.pi * rng.uniform(150, 300) * t) * (1 + np.sin(2 * np.pi * 3 * t)))
            wavfile.write(os.path.join(ds, spk, "audio", clip + ".wav"), 16000, speech.astype(np.int16))
            np.save(os.path.join(ds, spk, "video", clip + ".npy"), rng.integers(0, 256, (75, 128, 128), dtype=np.uint8))
    noise = os.path.join(tmp, "noise")
    os.makedirs(noise)
    for k in range(n_noise):
        wavfile.write(os.path.join(noise, "n%d.wav" % k), 16000, rng.normal(0, 2000, 20000 + 997 * k).astype(np.int16))
    return ds, noise


def run(args, cwd):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "speech_enhancer.py")] + args, cwd=cwd,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cli_preprocess_train_predict(gpu, tmp_path):
    tmp = str(tmp_path)
    ds, noise = make_dataset(tmp)
    base = os.path.join(tmp, "base")
    os.makedirs(base)
    out = run(["-bd", base, "preprocess", "-dn", "d", "-ds", ds, "-n", noise], tmp)
    assert "preprocessed 1 samples" in out
    run(["-bd", base, "train", "-mn", "m", "-tdn", "d", "-vdn", "d", "--init-only"], tmp)
    assert os.path.exists(os.path.join(base, "cache", "models", "m", "model.safetensors"))
    out = run(["-bd", base, "predict", "-mn", "m", "-dn", "d"], tmp)
    assert "loss:" in out
    enhanced = glob.glob(os.path.join(base, "out", "m", "d", "*", "*", "*", "enhanced.wav"))
    assert len(enhanced) == 1
    from scipy.io import wavfile
    sr, y = wavfile.read(enhanced[0])
    assert sr == 16000 and y.shape == (160 * (300 - 1),)
    for f in ("mixture.wav", "source.wav", "noise.wav"):
        assert os.path.exists(os.path.join(os.path.dirname(enhanced[0]), f))


def test_cli_train_fits_checkpoints_and_predicts(gpu, tmp_path):
    """speech_enhancer.py:31-58 without --init-only: sample sets from the preprocessed blobs, the normaliser fitted
    and applied in place to the training AND validation video, the fit (checkpointed every epoch to the model file),
    the final save — then predict runs on the trained model."""
    from avse_amd.model import KerasModel
    tmp = str(tmp_path)
    ds, noise = make_dataset(tmp)
    base = os.path.join(tmp, "base")
    os.makedirs(base)
    run(["-bd", base, "preprocess", "-dn", "d", "-ds", ds, "-n", noise], tmp)
    out = run(["-bd", base, "train", "-mn", "m", "-tdn", "d", "-vdn", "d", "--epochs", "2", "--seed", "1"], tmp)
    assert "epoch 2:" in out and "val_loss" in out
    model_dir = os.path.join(base, "cache", "models", "m")
    assert os.path.exists(os.path.join(model_dir, "normalization.npz"))
    trained = KerasModel.load(os.path.join(model_dir, "model.safetensors"))
    init = KerasModel.init(seed=1)
    assert not np.array_equal(trained.to_blob(), init.to_blob())       # the fit moved the parameters
    out = run(["-bd", base, "predict", "-mn", "m", "-dn", "d"], tmp)
    assert "loss:" in out
    assert len(glob.glob(os.path.join(base, "out", "m", "d", "*", "*", "*", "enhanced.wav"))) == 1


def test_cli_batched_predict_equals_per_sample(gpu, tmp_path):
    """predict's batched path (BatchPredictor: one forward over every sample's slices, one STFT / ISTFT of the stacked
    mixtures) writes the same wav files, bit for bit, and prints the same losses as the per-sample path
    (--per-sample: speech_enhancer.py:61-88's loop, one sample per forward)."""
    tmp = str(tmp_path)
    ds, noise = make_dataset(tmp, n_noise=4)
    base = os.path.join(tmp, "base")
    os.makedirs(base)
    out = run(["-bd", base, "preprocess", "-dn", "d", "-ds", ds, "-n", noise], tmp)
    assert "preprocessed 4 samples" in out
    run(["-bd", base, "train", "-mn", "m", "-tdn", "d", "-vdn", "d", "--init-only"], tmp)
    results = {}
    for mode in ("batched", "per_sample"):
        extra = ["--per-sample"] if mode == "per_sample" else []
        out = run(["-bd", base, "predict", "-mn", "m", "-dn", "d"] + extra, tmp)
        losses = [ln for ln in out.splitlines() if ln.startswith("loss:")]
        assert len(losses) == 4, out
        run_dir = os.path.join(base, "out", "m", "d")
        wavs = sorted(glob.glob(os.path.join(run_dir, "*", "*", "*", "enhanced.wav")))
        assert len(wavs) == 4
        results[mode] = (losses, {os.path.join(*w.split(os.sep)[-3:]): open(w, "rb").read() for w in wavs})
        import shutil
        shutil.move(run_dir, run_dir + "_" + mode)
    assert results["batched"][0] == results["per_sample"][0]
    assert results["batched"][1].keys() == results["per_sample"][1].keys()
    for k in results["batched"][1]:
        assert results["batched"][1][k] == results["per_sample"][1][k], k
