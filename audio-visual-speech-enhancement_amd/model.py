"""Keras-layout parameter container for the network of /root/reference/network.py.

The layer table mirrors SpeechEnhancementNetwork's builders (network.py:88-175) with the shapes a
Keras build of `build((80, T), (128, 128, F))` produces (network.py:17-40): T = spectrogram frames per
200-ms slice (20 at 25 fps, 24 at 29.97 / 30 fps; data_processor.py:44-52), F = video frames per slice (5 at
25 / 29.97 fps, 6 at 30 fps; data_processor.py:24).  T sets the audio embedding (5 x ceil(T/4) x 128), the
concat width (+ 2048) and the dense widths (concat // 4, network.py:55); F is v_conv1's input channels.
`layers(T, F)` is that table; `LAYERS` the 25-fps one (build((80, 20), (128, 128, 5))).  Tensors keep Keras
layouts so a trained reference model maps 1:1 onto them:
    Conv2D           kernel (kh, kw, cin, cout)    bias (cout,)
    Conv2DTranspose  kernel (kh, kw, cout, cin)    bias (cout,)
    Dense            kernel (in, out)              bias (out,)
    BatchNormalization gamma, beta, moving_mean, moving_variance (C,)
`to_blob()` flattens them in the canonical order avse_weights_load (include/avse.h) expects.
"""
import json
from collections import OrderedDict, namedtuple

import numpy as np

Layer = namedtuple("Layer", "name kind cin cout kernel strides bn_channels ref")


def _ceil(a, b):
    return -(-a // b)


def embedding(T):
    """(audio embedding size, concat width, shared embedding size) of build((80, T), ...): network.py:47-55."""
    aemb = 5 * _ceil(_ceil(T, 2), 2) * 128
    cat = aemb + 2 * 2 * 512
    return aemb, cat, cat // 4


def shape_supported(T, F):
    """The shapes libavse implements (include/avse.h avse_weights_blob_floats_shape): the decoder reproduces 80 x T
    only for T a multiple of 4 (else Keras' own fit / evaluate would fail on the shape mismatch too)."""
    return T >= 4 and T % 4 == 0 and T <= 64 and 1 <= F <= 8   # csrc/netplan.h plan_valid


def layers(T=20, F=5):
    """(kind: conv | deconv | dense); bn_channels = 0 -> no BatchNormalization after the layer"""
    aemb, cat, emb = embedding(T)
    return (
    Layer("a_conv1", "conv", 1, 64, (5, 5), (2, 2), 64, "network.py:89"),
    Layer("a_conv2", "conv", 64, 64, (4, 4), (1, 1), 64, "network.py:93"),
    Layer("a_conv3", "conv", 64, 128, (4, 4), (2, 2), 128, "network.py:97"),
    Layer("a_conv4", "conv", 128, 128, (2, 2), (2, 1), 128, "network.py:101"),
    Layer("a_conv5", "conv", 128, 128, (2, 2), (2, 1), 128, "network.py:105"),
    Layer("v_conv1", "conv", F, 128, (5, 5), (1, 1), 128, "network.py:139"),
    Layer("v_conv2", "conv", 128, 128, (5, 5), (1, 1), 128, "network.py:145"),
    Layer("v_conv3", "conv", 128, 256, (3, 3), (1, 1), 256, "network.py:151"),
    Layer("v_conv4", "conv", 256, 256, (3, 3), (1, 1), 256, "network.py:157"),
    Layer("v_conv5", "conv", 256, 512, (3, 3), (1, 1), 512, "network.py:163"),
    Layer("v_conv6", "conv", 512, 512, (3, 3), (1, 1), 512, "network.py:169"),
    Layer("enc_dense", "dense", cat, emb, None, None, emb, "network.py:56"),
    Layer("dec_dense1", "dense", emb, emb, None, None, emb, "network.py:69"),
    Layer("dec_dense2", "dense", emb, aemb, None, None, 128, "network.py:75-78"),  # BN after Reshape(5,W,128)
    Layer("d_deconv1", "deconv", 128, 128, (2, 2), (2, 1), 128, "network.py:113"),
    Layer("d_deconv2", "deconv", 128, 128, (2, 2), (2, 1), 128, "network.py:117"),
    Layer("d_deconv3", "deconv", 128, 128, (4, 4), (2, 2), 128, "network.py:121"),
    Layer("d_deconv4", "deconv", 128, 64, (4, 4), (1, 1), 64, "network.py:125"),
    Layer("d_deconv5", "deconv", 64, 64, (5, 5), (2, 2), 64, "network.py:129"),
    Layer("d_deconv6", "deconv", 64, 1, (1, 1), (1, 1), 0, "network.py:133"),
    )


LAYERS = layers(20, 5)
AUDIO_SHAPE = (80, 20)          # data_processor.py:47-55 at 16 kHz / 25 fps
VIDEO_SHAPE = (128, 128, 5)     # data_processor.py:12, :24
BN_EPS = 1e-3
LRELU_ALPHA = 0.3
FORMAT = "avse-keras-layout-v1"


def kernel_shape(layer):
    if layer.kind == "dense":
        return (layer.cin, layer.cout)
    kh, kw = layer.kernel
    if layer.kind == "conv":
        return (kh, kw, layer.cin, layer.cout)
    return (kh, kw, layer.cout, layer.cin)


def tensor_names(T=20, F=5):
    """Canonical (name, shape) order of the weight blob of build((80, T), (128, 128, F))."""
    out = []
    for L in layers(T, F):
        out.append((L.name + "/kernel", kernel_shape(L)))
        out.append((L.name + "/bias", (L.cout,)))
        if L.bn_channels:
            for p in ("gamma", "beta", "moving_mean", "moving_variance"):
                out.append((L.name + "_bn/" + p, (L.bn_channels,)))
    return out


def blob_floats(T=20, F=5):
    return int(sum(int(np.prod(s)) for _, s in tensor_names(T, F)))


def shape_of(tensors):
    """(T, F) of a Keras-layout tensor dict: F = v_conv1's input channels, T from dec_dense2's output width."""
    F = int(tensors["v_conv1/kernel"].shape[2])
    aemb = int(tensors["dec_dense2/kernel"].shape[1])
    if aemb % 640:
        raise ValueError(f"dec_dense2 width {aemb} is not 5 x W x 128")
    return 4 * (aemb // 640), F


def _glorot_limit(shape):
    # keras.initializers._compute_fans (channels_last)
    if len(shape) == 2:
        fan_in, fan_out = shape
    else:
        rf = int(np.prod(shape[:-2]))
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    return np.sqrt(6.0 / (fan_in + fan_out))


class KerasModel:
    """Holds the network's Keras-layout tensors (float32), keyed 'layer/param'."""

    def __init__(self, tensors):
        for n in ("v_conv1/kernel", "dec_dense2/kernel"):
            if n not in tensors:
                raise ValueError(f"missing tensor {n}")
        self.T, self.F = shape_of(tensors)
        names = tensor_names(self.T, self.F)
        missing = [n for n, _ in names if n not in tensors]
        if missing:
            raise ValueError(f"missing tensors: {missing[:4]}...")
        for n, s in names:
            if tuple(tensors[n].shape) != tuple(s):
                raise ValueError(f"{n}: shape {tensors[n].shape}, expected {s}")
        self.tensors = OrderedDict((n, np.ascontiguousarray(tensors[n], dtype=np.float32)) for n, _ in names)

    @property
    def audio_shape(self):
        return (80, self.T)

    @property
    def video_shape(self):
        return (128, 128, self.F)

    # ---- construction -------------------------------------------------------------------
    @classmethod
    def init(cls, seed=0, randomize=False, audio_shape=AUDIO_SHAPE, video_shape=VIDEO_SHAPE):
        """Keras-default init (glorot_uniform kernels, zero bias, BN identity stats) of build(audio_shape, video_shape).

        randomize=True additionally draws non-trivial biases and BN statistics
        (gamma~U(0.5,1.5), beta~N(0,0.1), mean~N(0,0.1), var~U(0.5,1.5)) so
        that bias/BN folding is exercised by the parity tests."""
        if len(audio_shape) != 2 or audio_shape[0] != 80 or tuple(video_shape[:2]) != (128, 128):
            raise ValueError(f"network inputs are [80, T] x [128, 128, F], got {audio_shape} x {video_shape}")
        rng = np.random.default_rng(seed)
        t = OrderedDict()
        for L in layers(int(audio_shape[1]), int(video_shape[2])):
            ks = kernel_shape(L)
            lim = _glorot_limit(ks)
            t[L.name + "/kernel"] = rng.uniform(-lim, lim, size=ks).astype(np.float32)
            t[L.name + "/bias"] = (rng.normal(0, 0.05, size=(L.cout,)) if randomize else np.zeros(L.cout)).astype(np.float32)
            if L.bn_channels:
                C = L.bn_channels
                if randomize:
                    t[L.name + "_bn/gamma"] = rng.uniform(0.5, 1.5, C).astype(np.float32)
                    t[L.name + "_bn/beta"] = rng.normal(0, 0.1, C).astype(np.float32)
                    t[L.name + "_bn/moving_mean"] = rng.normal(0, 0.1, C).astype(np.float32)
                    t[L.name + "_bn/moving_variance"] = rng.uniform(0.5, 1.5, C).astype(np.float32)
                else:
                    t[L.name + "_bn/gamma"] = np.ones(C, np.float32)
                    t[L.name + "_bn/beta"] = np.zeros(C, np.float32)
                    t[L.name + "_bn/moving_mean"] = np.zeros(C, np.float32)
                    t[L.name + "_bn/moving_variance"] = np.ones(C, np.float32)
        return cls(t)

    # ---- views --------------------------------------------------------------------------
    def to_blob(self):
        return np.concatenate([self.tensors[n].ravel() for n, _ in tensor_names()]).astype(np.float32)

    @classmethod
    def from_blob(cls, blob, T=20, F=5):
        """Inverse of to_blob (the canonical layout of include/avse.h avse_weights_load[_shape])."""
        blob = np.asarray(blob, dtype=np.float32).ravel()
        t, off = OrderedDict(), 0
        for n, shape in tensor_names(T, F):
            k = int(np.prod(shape))
            t[n] = blob[off:off + k].reshape(shape).copy()
            off += k
        if off != blob.size:
            raise ValueError(f"blob has {blob.size} floats, the network {off}")
        return cls(t)

    def layer_dict(self):
        """{'a_conv1': {'kernel', 'bias'}, 'a_conv1_bn': {'gamma', ...}, ...}"""
        d = {}
        for n, a in self.tensors.items():
            layer, p = n.split("/")
            d.setdefault(layer, {})[p] = a
        return d

    # ---- persistence (safetensors; Keras HDF5 import is a converter) -----------
    def save(self, path):
        from safetensors.numpy import save_file
        save_file(dict(self.tensors), path, metadata={"format": FORMAT, "layers": json.dumps([L.name for L in LAYERS]),
                                                      "audio_shape": json.dumps(self.audio_shape),
                                                      "video_shape": json.dumps(self.video_shape)})

    @classmethod
    def load(cls, path):
        with open(path, "rb") as f:
            head = f.read(8)
        if head.startswith(b"\x89HDF"):
            raise ValueError(f"{path} is a Keras HDF5 model; convert it with tools/keras_h5_to_avse.py first")
        from safetensors.numpy import load_file
        return cls(load_file(path))
