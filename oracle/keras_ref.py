"""Keras-semantics restatement of the AVSE network forward pass — TEST INFRASTRUCTURE ONLY.

Restates `/root/reference/network.py` (Keras >= 2.0.4 with the TF backend, README.md:14) in
PyTorch-CPU ops, in float64 (the truth the HIP path is compared against) or float32 (the
"Keras-CPU fp32" behaviour, also used as bench.py's cpu_baseline leg).

Keras semantics restated here (Keras 2.0 defaults):
  * Conv2D(padding='same')  — TF 'SAME': out = ceil(in/s), pad_total = max((out-1)*s + k - in, 0),
    pad_before = pad_total // 2 (the extra pixel goes bottom/right).
  * Conv2DTranspose('same') — TF conv2d_transpose to out = in*s: full transposed conv (no kernel
    flip) cropped at pad_before = max(k - s, 0) // 2.  Kernel layout (kh, kw, out, in).
  * BatchNormalization      — inference: (x - mean) / sqrt(var + 1e-3) * gamma + beta.
  * LeakyReLU               — alpha = 0.3.
  * MaxPooling2D(2, 2, 'same') on even sizes; Dropout = identity at inference.
  * Flatten                 — NHWC row-major; concatenate([audio, video]) audio first (network.py:53).
"""
import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-3
LRELU_ALPHA = 0.3

# Layer spec restated from network.py (name, kind, filters, kernel, strides, has_bn, pool, line).
AUDIO_ENCODER = [
    ("a_conv1", "conv", 64, (5, 5), (2, 2), True, False, "network.py:89"),
    ("a_conv2", "conv", 64, (4, 4), (1, 1), True, False, "network.py:93"),
    ("a_conv3", "conv", 128, (4, 4), (2, 2), True, False, "network.py:97"),
    ("a_conv4", "conv", 128, (2, 2), (2, 1), True, False, "network.py:101"),
    ("a_conv5", "conv", 128, (2, 2), (2, 1), True, False, "network.py:105"),
]
VIDEO_ENCODER = [
    ("v_conv1", "conv", 128, (5, 5), (1, 1), True, True, "network.py:139"),
    ("v_conv2", "conv", 128, (5, 5), (1, 1), True, True, "network.py:145"),
    ("v_conv3", "conv", 256, (3, 3), (1, 1), True, True, "network.py:151"),
    ("v_conv4", "conv", 256, (3, 3), (1, 1), True, True, "network.py:157"),
    ("v_conv5", "conv", 512, (3, 3), (1, 1), True, True, "network.py:163"),
    ("v_conv6", "conv", 512, (3, 3), (1, 1), True, True, "network.py:169"),
]
AUDIO_DECODER = [
    ("d_deconv1", "deconv", 128, (2, 2), (2, 1), True, False, "network.py:113"),
    ("d_deconv2", "deconv", 128, (2, 2), (2, 1), True, False, "network.py:117"),
    ("d_deconv3", "deconv", 128, (4, 4), (2, 2), True, False, "network.py:121"),
    ("d_deconv4", "deconv", 64, (4, 4), (1, 1), True, False, "network.py:125"),
    ("d_deconv5", "deconv", 64, (5, 5), (2, 2), True, False, "network.py:129"),
    ("d_deconv6", "deconv", 1, (1, 1), (1, 1), False, False, "network.py:133"),
]


def _t(a, dtype):
    return torch.as_tensor(np.asarray(a), dtype=dtype)


def _same_pads(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


def conv_same(x, kernel, bias, strides, dtype):
    """x NCHW; kernel keras (kh, kw, cin, cout)."""
    kh, kw = kernel.shape[:2]
    pt, pb = _same_pads(x.shape[2], kh, strides[0])
    pl, pr = _same_pads(x.shape[3], kw, strides[1])
    x = F.pad(x, (pl, pr, pt, pb))
    w = _t(kernel, dtype).permute(3, 2, 0, 1).contiguous()
    return F.conv2d(x, w, _t(bias, dtype), stride=tuple(strides))


def deconv_same(x, kernel, bias, strides, dtype):
    """x NCHW; kernel keras (kh, kw, cout, cin)."""
    kh, kw = kernel.shape[:2]
    H, W = x.shape[2], x.shape[3]
    w = _t(kernel, dtype).permute(3, 2, 0, 1).contiguous()   # (cin, cout, kh, kw)
    y = F.conv_transpose2d(x, w, _t(bias, dtype), stride=tuple(strides))
    pt = max(kh - strides[0], 0) // 2
    pl = max(kw - strides[1], 0) // 2
    return y[:, :, pt:pt + H * strides[0], pl:pl + W * strides[1]]


def bn(x, p, dtype, channel_dim=1):
    shape = [1] * x.dim()
    shape[channel_dim] = -1
    g, b, m, v = (_t(p[k], dtype).reshape(shape) for k in ("gamma", "beta", "moving_mean", "moving_variance"))
    return (x - m) / torch.sqrt(v + BN_EPS) * g + b


def lrelu(x):
    return torch.where(x >= 0, x, LRELU_ALPHA * x)


def forward(weights, mixed_spectrograms, video_samples, dtype=torch.float64, threads=None, intermediates=None):
    """network.py:208-212 predict without the squeeze: returns [N, 80, 20] numpy.

    weights: dict name -> dict of Keras-layout arrays ('kernel', 'bias'; BN layers under
    name + '_bn' with gamma/beta/moving_mean/moving_variance).
    mixed_spectrograms [N, 80, T]; video_samples [N, 128, 128, F] (already normalised), or None for an
    all-zero video input (BASELINE configs[2]): the video branch then runs once on one zero clip and its
    embedding is shared by every clip, which is what a zero batch computes clip by clip.
    intermediates: optional dict, filled with each layer's NHWC output (after BN/LReLU/pool).
    """
    def keep(name, t):
        if intermediates is not None:
            intermediates[name] = (t.permute(0, 2, 3, 1) if t.dim() == 4 else t).numpy().copy()

    if threads is not None:
        torch.set_num_threads(threads)
    with torch.no_grad():
        a = _t(mixed_spectrograms, dtype)[:, None, :, :]          # expand_dims(-1) -> NCHW, C=1
        if video_samples is None:
            video_samples = np.zeros((1, 128, 128, weights["v_conv1"]["kernel"].shape[2]), np.float32)
        v = _t(video_samples, dtype).permute(0, 3, 1, 2)           # NHWC -> NCHW
        for name, kind, f, k, s, has_bn, pool, _ in AUDIO_ENCODER:
            a = lrelu(bn(conv_same(a, weights[name]["kernel"], weights[name]["bias"], s, dtype), weights[name + "_bn"], dtype))
            keep(name, a)
        for name, kind, f, k, s, has_bn, pool, _ in VIDEO_ENCODER:
            v = lrelu(bn(conv_same(v, weights[name]["kernel"], weights[name]["bias"], s, dtype), weights[name + "_bn"], dtype))
            v = F.max_pool2d(v, 2, 2)
            keep(name, v)
        N = a.shape[0]
        a_emb_shape = a.shape[1:]
        vflat = v.permute(0, 2, 3, 1).reshape(v.shape[0], -1)
        if vflat.shape[0] != N:                                     # the shared all-zero-video embedding
            vflat = vflat.expand(N, -1)
        x = torch.cat([a.permute(0, 2, 3, 1).reshape(N, -1), vflat], dim=1)
        keep("concat", x)
        x = lrelu(bn(x @ _t(weights["enc_dense"]["kernel"], dtype) + _t(weights["enc_dense"]["bias"], dtype), weights["enc_dense_bn"], dtype))
        keep("enc_dense", x)
        x = lrelu(bn(x @ _t(weights["dec_dense1"]["kernel"], dtype) + _t(weights["dec_dense1"]["bias"], dtype), weights["dec_dense1_bn"], dtype))
        keep("dec_dense1", x)
        x = x @ _t(weights["dec_dense2"]["kernel"], dtype) + _t(weights["dec_dense2"]["bias"], dtype)
        C, H, W = a_emb_shape
        x = x.reshape(N, H, W, C)                                   # Reshape(audio_embedding_shape), NHWC
        x = lrelu(bn(x, weights["dec_dense2_bn"], dtype, channel_dim=3)).permute(0, 3, 1, 2)
        keep("dec_dense2", x)
        for name, kind, f, k, s, has_bn, pool, _ in AUDIO_DECODER:
            x = deconv_same(x, weights[name]["kernel"], weights[name]["bias"], s, dtype)
            if has_bn:
                x = lrelu(bn(x, weights[name + "_bn"], dtype))
            keep(name, x)
        return x[:, 0].numpy()


def mse(pred, target):
    """network.py:214-220 evaluate: Keras 'mean_squared_error' averaged over every element."""
    pred = np.asarray(pred, dtype=np.float64)
    target = np.asarray(target, dtype=np.float64)
    return float(np.mean((pred - target) ** 2))
