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


def check_gradients(g, ref_g, tol=1e-2):
    """Every gradient tensor within relative RMS `tol` of the reference.  Tensors whose reference gradient is zero
    (exactly, in float64: at N = 1 the dense layers' BatchNormalization sees one sample, its batch variance is 0 and
    it passes no gradient back, so the whole encoder's gradient vanishes) and the pre-BN biases (see pre_bn_bias)
    must stay below 1e-6 resp. 1e-3 of the largest gradient RMS of the network."""
    rms = {n: float(np.sqrt(np.mean(np.asarray(r, np.float64) ** 2))) for n, r in ref_g.items()}
    top = max(rms.values())
    bad = {}
    for name, ref in ref_g.items():
        if name.endswith(("moving_mean", "moving_variance")):
            assert not np.any(g[name]), name
            continue
        got_rms = float(np.sqrt(np.mean(g[name].astype(np.float64) ** 2)))
        if pre_bn_bias(name):
            scale = max(rms[name.replace("/bias", "/kernel")], 1e-3 * top)
            if got_rms > 1e-3 * scale:
                bad[name] = "pre-BN bias gradient not ~0"
            continue
        if rms[name] <= 1e-12 * top:
            if got_rms > 1e-6 * top:
                bad[name] = f"reference gradient is zero, device RMS {got_rms:.3e}"
            continue
        e = rel_rms(g[name], ref)
        print(f"{name:28s} rel RMS {e:.2e}")
        if e > tol:
            bad[name] = e
    assert not bad, sorted(bad.items())


# N = 16 with max_batch = 16 is the reference's fit batch (network.py:203) and the shape bench.py's train leg times
# (wg_splits, rows_per_split, k_wgrad_nat splits and the column-reduction blocks all change with N); N = 1: the dense
# layers' BatchNormalization over a single sample (variance 0)
@pytest.mark.parametrize("N,rate,max_batch", [(4, 0.25, 8), (3, 0.0, 8), (16, 0.25, 16), (1, 0.0, 16)])
def test_gradients_match_oracle(gpu, N, rate, max_batch):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=21, randomize=True)
    rng = np.random.default_rng(5 + N)
    mel, video, target = batch(rng, N)
    tr = ops.Trainer(model, max_batch=max_batch, device=gpu)
    loss = float(tr.step(*_dev(gpu, mel, video, target), dropout=rate, seed=1234, grads_only=True).item())
    g = tr.gradients()
    ref_loss, ref_g, stats = KT.gradients(model.tensors, mel, video, target, rate=rate, seed=1234)
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    check_gradients(g, ref_g)
    # moving statistics were updated by the training-mode forward
    new = tr.model().tensors
    for name, ref in KT.moving_stats(model.tensors, stats).items():
        assert rel_rms(new[name], ref) <= 1e-5, name


def test_max_batch_1023_equals_repeated_small_batch(gpu):
    """The trainer's largest batch (max_batch 1023, the int32-indexing cap of include/avse.h) through a
    size-independent property: a batch of 3 clips repeated k times has the same batch statistics, the same mean
    loss and the same gradients for every k (no dropout).
      * k = 341 (N = 1023) against k = 2 (N = 6): relative 1e-2 (measured 3.7e-3 at most, profiles/r03c_gputest.log;
        d_deconv5's kernel gradient agrees to 5.7e-6, so the per-row arithmetic is identical and what remains is
        fp32 column sums over 1.6M instead of 9,600 rows, amplified where a BN gradient sum cancels);
      * against the float64 oracle at N = 3: 2e-2.  Measured (profiles/r03b_train_bisect.log, tools/train_bisect.py):
        every k from 2 to 341 lands at the SAME 8.9e-3 on d_deconv5/kernel (1.4e-2 upstream) against the N = 3 step,
        and N = 3 itself at ~0 — the signature of one LeakyReLU slope flip at a d_deconv5 BN output within fp32
        rounding of zero (the batch statistics of 6 rows round differently from those of 3), not of an
        accumulation error, which would grow with k.  The standard 1e-2 gate of the distinct-clip tests holds
        for them (N = 1, 3, 4, 16 above)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=23, randomize=True)
    mel, video, target = batch(np.random.default_rng(31), 3)

    def step(k):
        rep = [np.ascontiguousarray(np.tile(a, (k,) + (1,) * (a.ndim - 1))) for a in (mel, video, target)]
        tr = ops.Trainer(model, max_batch=3 * k, device=gpu)
        loss = float(tr.step(*_dev(gpu, *rep), dropout=0.0, grads_only=True).item())
        g = tr.gradients()
        del tr
        torch.cuda.empty_cache()
        return loss, g

    l6, g6 = step(2)
    l1023, g1023 = step(341)
    assert np.isfinite(l1023) and abs(l1023 - l6) <= 1e-5 * abs(l6), (l1023, l6)
    print("N = 1023 vs N = 6")
    check_gradients(g1023, g6, tol=1e-2)
    ref_loss, ref_g, _ = KT.gradients(model.tensors, mel, video, target, rate=0.0, seed=0)
    assert abs(l1023 - ref_loss) <= 1e-5 * abs(ref_loss), (l1023, ref_loss)
    print("N = 1023 vs float64 oracle (N = 3)")
    check_gradients(g1023, ref_g, tol=2e-2)


@pytest.mark.parametrize("N", [4, 16])
def test_adam_steps_match_oracle(gpu, N):
    """Three fit steps, at N = 4 and at the reference's fit batch of 16 (network.py:203).  Adam normalises each gradient element by its own running RMS, so its first steps are
    ~lr * sign(g): elements whose gradient is within float32 noise of zero move by +-lr on either side.  The
    update arithmetic is therefore checked on the device's own gradients (Keras 2.0 Adam restated in float64,
    every tensor, relative 5e-4 of the update: the float32 parameter itself rounds at ~1e-7 of a unit-size gamma
    against a 3-step update of ~1.5e-3), and the trajectory against the float64 oracle run end to end
    through the losses (relative 1e-3)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=3, randomize=True)
    rng = np.random.default_rng(77)
    batches = [batch(rng, N) + (100 + i,) for i in range(3)]
    tr = ops.Trainer(model, max_batch=N, device=gpu)
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
        p0 = model.tensors[name]
        d_got, d_ref = got[name].astype(np.float64) - p0, ref - p0
        # relative 5e-4 of the update, plus the rounding of the stored float32 parameter (half an ulp per step): the
        # biases of the dense layers before BatchNormalization get gradients at float32 noise level (BN cancels a
        # bias), so at N = 16 their updates are a few ulps of the bias and the rounding is most of the difference
        ulp = np.spacing(np.abs(p0).astype(np.float32)).astype(np.float64)
        err = float(np.sqrt(np.mean((d_got - d_ref) ** 2)))
        bound = 5e-4 * float(np.sqrt(np.mean(d_ref ** 2))) + 1.5 * float(np.sqrt(np.mean(ulp ** 2)))
        if err > bound:
            bad[name] = (err, bound, rel_rms(d_got, d_ref))
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
