"""Training step parity (network.py:177-206): libavse's fp32 Keras fit step (csrc/train.hip)
against the float64 autograd restatement of Keras 2.0 training semantics (oracle/keras_train_ref.py).

Tolerances (float32 device arithmetic against float64 autograd through 20 layers of batch-statistics BN):
  * loss: relative 1e-5;
  * every gradient tensor: relative RMS <= 1e-2 — torch-CPU float32 itself lands at 1e-5..4e-3 against float64
    (v_conv1 / v_conv2 reduce over 65k-262k pixels), and an element whose BN output sits within float32 rounding
    of zero takes the other LeakyReLU slope (measured: one such pixel of d_deconv5 moves every upstream gradient
    by ~1.5e-3); a wrong tap, channel or mask shows up as O(1) — except the biases of layers followed by
    BatchNormalization,
    whose true gradient is exactly zero (BN removes the batch mean): there the float32 sum over the batch's pixels
    must stay below 1e-3 x the RMS of the same layer's kernel gradient;
  * BN moving statistics after the step: relative 1e-5;
  * three Adam steps: the update arithmetic on the device's own gradients (relative 5e-4), the loss trajectory
    against the oracle's (relative 1e-3).
"""
import numpy as np
import pytest
import torch

from oracle import keras_train_ref as KT

pytestmark = pytest.mark.gpu


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-300))


def batch(rng, N):
    mel = rng.normal(-40, 12, (N, 80, 20)).astype(np.float32)
    video = rng.normal(0, 1, (N, 128, 128, 5)).astype(np.float32)      # normalised crops
    target = (mel + rng.normal(0, 3, mel.shape)).astype(np.float32)
    return mel, video, target


def pre_bn_bias(name):
    """Biases whose true gradient is zero: a BatchNormalization over the same channels follows the layer.
    (dec_dense2's bias is per feature of the 3200-vector, its BN per channel of the Reshape: not zero.)"""
    layer = name.split("/")[0]
    return name.endswith("/bias") and layer not in ("d_deconv6", "dec_dense2")


def _dev(gpu, *arrays):
    return [torch.from_numpy(a).to(gpu) for a in arrays]


@pytest.mark.parametrize("N,rate", [(4, 0.25), (3, 0.0)])
def test_gradients_match_oracle(gpu, N, rate):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=21, randomize=True)
    rng = np.random.default_rng(5 + N)
    mel, video, target = batch(rng, N)
    tr = ops.Trainer(model, max_batch=8, device=gpu)
    loss = float(tr.step(*_dev(gpu, mel, video, target), dropout=rate, seed=1234, grads_only=True).item())
    g = tr.gradients()
    ref_loss, ref_g, stats = KT.gradients(model.tensors, mel, video, target, rate=rate, seed=1234)
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    bad = {}
    for name, ref in ref_g.items():
        if name.endswith(("moving_mean", "moving_variance")):
            assert not np.any(g[name]), name
            continue
        if pre_bn_bias(name):
            scale = np.sqrt(np.mean(ref_g[name.replace("/bias", "/kernel")] ** 2))
            if np.sqrt(np.mean(g[name].astype(np.float64) ** 2)) > 1e-3 * scale:
                bad[name] = "pre-BN bias gradient not ~0"
            continue
        e = rel_rms(g[name], ref)
        print(f"{name:28s} rel RMS {e:.2e}")
        if e > 1e-2:
            bad[name] = e
    assert not bad, sorted(bad.items())
    # moving statistics were updated by the training-mode forward
    new = tr.model().tensors
    for name, ref in KT.moving_stats(model.tensors, stats).items():
        assert rel_rms(new[name], ref) <= 1e-5, name


def test_adam_steps_match_oracle(gpu):
    """Three fit steps.  Adam normalises each gradient element by its own running RMS, so its first steps are
    ~lr * sign(g): elements whose gradient is within float32 noise of zero move by +-lr on either side.  The
    update arithmetic is therefore checked on the device's own gradients (Keras 2.0 Adam restated in float64,
    every tensor, relative 5e-4 of the update: the float32 parameter itself rounds at ~1e-7 of a unit-size gamma
    against a 3-step update of ~1.5e-3), and the trajectory against the float64 oracle run end to end
    through the losses (relative 1e-3)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=3, randomize=True)
    rng = np.random.default_rng(77)
    batches = [batch(rng, 4) + (100 + i,) for i in range(3)]
    tr = ops.Trainer(model, max_batch=4, device=gpu)
    params = {n: a.astype(np.float64) for n, a in model.tensors.items()}
    m = {n: np.zeros_like(a) for n, a in params.items()}
    v = {n: np.zeros_like(a) for n, a in params.items()}
    losses = []
    for t, (mel, video, target, seed) in enumerate(batches, start=1):
        losses.append(float(tr.step(*_dev(gpu, mel, video, target), lr=5e-4, dropout=0.25, seed=seed).item()))
        KT.adam_step(params, tr.gradients(), m, v, t, 5e-4)
    assert tr.iterations == 3
    got = tr.model().tensors
    bad = {}
    for name, ref in params.items():
        if name.endswith(("moving_mean", "moving_variance")):
            continue
        e = rel_rms(got[name].astype(np.float64) - model.tensors[name], ref - model.tensors[name])
        if e > 5e-4:
            bad[name] = e
    assert not bad, sorted(bad.items())
    _, ref_losses = KT.train_steps(model.tensors, batches, lr=5e-4, rate=0.25)
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-3)


def test_fit_reduces_loss_and_checkpoints(gpu, tmp_path):
    """network.train (Keras fit loop) on a small fixed set: training loss falls, a checkpoint is written."""
    from avse_amd.network import SpeechEnhancementNetwork
    rng = np.random.default_rng(9)
    mel, video, target = batch(rng, 24)
    net = SpeechEnhancementNetwork.build((80, 20), (128, 128, 5), seed=2)
    path = str(tmp_path / "model.safetensors")
    hist = net.train(mel[:16], video[:16], target[:16], mel[16:], video[16:], target[16:], path,
                     batch_size=8, epochs=4, verbose=0)
    assert len(hist) == 4
    assert hist[-1]["loss"] < hist[0]["loss"]
    reloaded = SpeechEnhancementNetwork.load(path)
    assert np.array_equal(reloaded.model.to_blob(), net.model.to_blob())


def test_trainer_rejects_bad_batches(gpu):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    tr = ops.Trainer(KerasModel.init(seed=0), max_batch=2, device=gpu)
    mel, video, target = batch(np.random.default_rng(0), 3)
    with pytest.raises(ValueError):
        tr.step(*_dev(gpu, mel, video, target))
    with pytest.raises(ValueError):
        tr.step(*_dev(gpu, mel[:2], video[:1], target[:2]))
