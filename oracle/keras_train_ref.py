"""Keras-2.0 training-step restatement of SpeechEnhancementNetwork.train — TEST INFRASTRUCTURE ONLY.

`/root/reference/network.py:177-206` trains with `Model.fit(batch_size=16)` on the model compiled at network.py:35-36
(`optimizers.adam(lr=5e-4)`, `loss='mean_squared_error'`).  Keras is not importable here, so its published
training-mode semantics are restated in float64 PyTorch-CPU autograd (parity unpinned against Keras itself):

  * BatchNormalization(momentum=0.99, epsilon=1e-3), learning phase 1: normalise with the batch mean and the biased
    batch variance (tf.nn.moments) over every axis but the channel; moving_mean / moving_variance <-
    m * 0.99 + batch * 0.01 (K.moving_average_update, Keras 2.0.x: no sample-size correction);
  * Dropout(0.25) after every video MaxPooling2D (network.py:142-174): kept values scaled by 1 / (1 - rate).  The
    mask is the product's counter-based hash (csrc/train.hip drop_hash), restated bit-exactly in numpy below so
    both sides drop the same elements;
  * mean_squared_error averaged over every element;
  * Adam (Keras 2.0.x optimizers.py): t += 1, lr_t = lr sqrt(1 - b2^t) / (1 - b1^t), m = b1 m + (1 - b1) g,
    v = b2 v + (1 - b2) g^2, p -= lr_t m / (sqrt(v) + 1e-8).
Layer geometry (TF 'SAME' padding, transposed-conv crop, HWC flatten, audio-first concat) is keras_ref's.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import keras_ref as K

BN_MOMENTUM = 0.99
LAYER_INDEX = {name: i for i, name in enumerate(
    [n for n, *_ in K.AUDIO_ENCODER] + [n for n, *_ in K.VIDEO_ENCODER] + ["enc_dense", "dec_dense1", "dec_dense2"]
    + [n for n, *_ in K.AUDIO_DECODER])}


def drop_hash(seed, layer, idx):
    """csrc/train.hip drop_hash, uint32 arithmetic (numpy wraps on overflow)."""
    with np.errstate(over="ignore"):
        idx = np.asarray(idx, dtype=np.uint32)
        h = idx * np.uint32(0x9E3779B1) ^ (np.uint32(seed) * np.uint32(0x85EBCA77) + np.uint32(layer) * np.uint32(0xC2B2AE3D))
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x7FEB352D)
        h ^= h >> np.uint32(15)
        h *= np.uint32(0x846CA68B)
        h ^= h >> np.uint32(16)
    return h


def dropout_scale(seed, layer, shape_nhwc, rate):
    """Per-element multiplier (0 or 1 / (1 - rate)) for a layer output of NHWC shape."""
    if rate <= 0:
        return np.ones(shape_nhwc)
    h = drop_hash(seed, layer, np.arange(int(np.prod(shape_nhwc)), dtype=np.uint64).astype(np.uint32))
    u = (h >> np.uint32(8)).astype(np.float64) * (1.0 / 16777216.0)
    return np.where(u >= rate, 1.0 / (1.0 - rate), 0.0).reshape(shape_nhwc)


def _bn_train(x, gamma, beta, channel_dim, stats, name):
    dims = [d for d in range(x.dim()) if d != channel_dim]
    mean = x.mean(dim=dims, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=dims, keepdim=True)
    stats[name] = (mean.detach().double().flatten().numpy().copy(), var.detach().double().flatten().numpy().copy())
    shape = [1] * x.dim()
    shape[channel_dim] = -1
    return (x - mean) / torch.sqrt(var + K.BN_EPS) * gamma.reshape(shape) + beta.reshape(shape)


def train_forward(p, mel, video, target, rate, seed, stats, dt=torch.float64):
    """p: {tensor name: leaf tensor of dtype dt}; video already normalised.  Returns the scalar MSE."""
    a = torch.as_tensor(np.asarray(mel), dtype=dt)[:, None]
    v = torch.as_tensor(np.asarray(video), dtype=dt).permute(0, 3, 1, 2)

    def conv(x, name, s):
        kh, kw = p[name + "/kernel"].shape[:2]
        pt, pb = K._same_pads(x.shape[2], kh, s[0])
        pl, pr = K._same_pads(x.shape[3], kw, s[1])
        return F.conv2d(F.pad(x, (pl, pr, pt, pb)), p[name + "/kernel"].permute(3, 2, 0, 1), p[name + "/bias"], stride=s)

    def deconv(x, name, s):
        kh, kw = p[name + "/kernel"].shape[:2]
        H, W = x.shape[2], x.shape[3]
        y = F.conv_transpose2d(x, p[name + "/kernel"].permute(3, 2, 0, 1), p[name + "/bias"], stride=s)
        pt, pl = max(kh - s[0], 0) // 2, max(kw - s[1], 0) // 2
        return y[:, :, pt:pt + H * s[0], pl:pl + W * s[1]]

    def bn(x, name, channel_dim=1):
        return _bn_train(x, p[name + "_bn/gamma"], p[name + "_bn/beta"], channel_dim, stats, name)

    for name, _, _, _, s, _, _, _ in K.AUDIO_ENCODER:
        a = K.lrelu(bn(conv(a, name, s), name))
    for name, _, _, _, s, _, _, _ in K.VIDEO_ENCODER:
        v = F.max_pool2d(K.lrelu(bn(conv(v, name, s), name)), 2, 2)
        nhwc = (v.shape[0], v.shape[2], v.shape[3], v.shape[1])
        mask = torch.as_tensor(dropout_scale(seed, LAYER_INDEX[name], nhwc, rate), dtype=dt).permute(0, 3, 1, 2)
        v = v * mask
    N = a.shape[0]
    C, H, W = a.shape[1:]
    x = torch.cat([a.permute(0, 2, 3, 1).reshape(N, -1), v.permute(0, 2, 3, 1).reshape(N, -1)], dim=1)
    x = K.lrelu(bn(x @ p["enc_dense/kernel"] + p["enc_dense/bias"], "enc_dense"))
    x = K.lrelu(bn(x @ p["dec_dense1/kernel"] + p["dec_dense1/bias"], "dec_dense1"))
    x = (x @ p["dec_dense2/kernel"] + p["dec_dense2/bias"]).reshape(N, H, W, C)
    x = K.lrelu(bn(x, "dec_dense2", channel_dim=3)).permute(0, 3, 1, 2)
    for name, _, _, _, s, has_bn, _, _ in K.AUDIO_DECODER:
        x = deconv(x, name, s)
        if has_bn:
            x = K.lrelu(bn(x, name))
    y = x[:, 0]
    return ((y - torch.as_tensor(np.asarray(target), dtype=dt)) ** 2).mean()


def gradients(tensors, mel, video, target, rate=0.25, seed=0, dtype=torch.float64):
    """One training-mode forward + backward.  tensors: {name: array} (KerasModel.tensors).
    Returns (loss, {name: gradient} for the trainable tensors, {name: (batch mean, batch var)} per BN layer)."""
    p = {n: torch.tensor(np.asarray(a, dtype=np.float64), dtype=dtype,
                         requires_grad=not n.endswith(("moving_mean", "moving_variance")))
         for n, a in tensors.items()}
    stats = {}
    loss = train_forward(p, mel, video, target, rate, seed, stats, dtype)
    loss.backward()
    grads = {n: (t.grad.double().numpy().copy() if t.grad is not None else np.zeros(t.shape)) for n, t in p.items()}
    return float(loss.detach()), grads, stats


def moving_stats(tensors, stats):
    """The BN moving-average updates of one step: {name: new array} for every moving_mean / moving_variance."""
    out = {}
    for name, (mean, var) in stats.items():
        out[name + "_bn/moving_mean"] = np.asarray(tensors[name + "_bn/moving_mean"], np.float64) * BN_MOMENTUM + mean * (1 - BN_MOMENTUM)
        out[name + "_bn/moving_variance"] = (np.asarray(tensors[name + "_bn/moving_variance"], np.float64) * BN_MOMENTUM
                                             + var * (1 - BN_MOMENTUM))
    return out


def adam_step(params, grads, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """Keras 2.0 Adam on {name: array} dicts, t = iterations after this update (1 for the first).  In place."""
    lr_t = lr * np.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
    for n in params:
        if n.endswith(("moving_mean", "moving_variance")):
            continue
        g = grads[n]
        m[n] = b1 * m[n] + (1 - b1) * g
        v[n] = b2 * v[n] + (1 - b2) * g * g
        params[n] = params[n] - lr_t * m[n] / (np.sqrt(v[n]) + eps)
    return params


def train_steps(tensors, batches, lr=5e-4, rate=0.25):
    """Run len(batches) fit steps; batches = [(mel, video, target, seed)].  Returns (params, losses)."""
    params = {n: np.asarray(a, np.float64).copy() for n, a in tensors.items()}
    m = {n: np.zeros_like(a) for n, a in params.items()}
    v = {n: np.zeros_like(a) for n, a in params.items()}
    losses = []
    for t, (mel, video, target, seed) in enumerate(batches, start=1):
        loss, grads, stats = gradients(params, mel, video, target, rate, seed)
        losses.append(loss)
        params.update(moving_stats(params, stats))
        adam_step(params, grads, m, v, t, lr)
    return params, losses
