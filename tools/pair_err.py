"""CPU emulation of AVSE_F32_SPLIT's STORAGE error: the float64 oracle forward (oracle/keras_ref.py semantics) with
every materialised activation (and the two network inputs, which the kernels split on load) rounded the way the split
dtype stores it, products exact.  So the schemes differ only in how activations and weights are represented:

    fp32        activations and weights rounded to float32 (the exact-fp32 path's storage)
    pair        activations as the f16 pair h + l (h = f16(x), l = f16(x - h)), weights as per-output-channel
                power-of-two scaled pairs (csrc/capi.hip build_layer)
    pair+sigma  the same with a per-layer power-of-two activation scale 2^sigma_L (include/avse.h: the stored pair is
                of x 2^sigma_L; sigma from the BN statistics, capi.hip act_exponents)

Also prints each layer's activation magnitude (RMS, max) and the fraction of values whose lo piece is an f16
subnormal (|x| 2^sigma < 2^-3).

    python tools/pair_err.py [N] [seed] [db|plain] [trained|init]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd.model import KerasModel  # noqa: E402
from oracle import keras_ref as K  # noqa: E402
from oracle import librosa_ref as R  # noqa: E402
from conftest import synth_audio, synth_video  # noqa: E402

F64 = torch.float64


def q_fp32(x, sigma=0):
    return x.to(torch.float32).to(F64)


def q_pair(x, sigma=0):
    s = 2.0 ** sigma
    y = x * s
    h = y.to(torch.float16).to(F64)
    l = (y - h).to(torch.float16).to(F64)
    return (h + l) / s


def q_w_pair(w, axis_out):
    """per-output-channel scaled weight pair (build_layer): max |w| 2^e in [2^14, 2^15)"""
    w = torch.as_tensor(np.asarray(w, np.float32), dtype=F64)
    red = [d for d in range(w.dim()) if d != axis_out]
    mx = w.abs().amax(dim=red, keepdim=True)
    e = torch.where(mx > 0, 15 - torch.floor(torch.log2(mx)) - 1, torch.zeros_like(mx))
    s = 2.0 ** e
    y = w * s
    h = y.to(torch.float16).to(F64)
    l = (y - h).to(torch.float16).to(F64)
    return ((h + l) / s).numpy()


def act_exponents(wd, target=6.0):
    """sigma_L per layer from the BN statistics (the data-free rule of capi.hip): the layer's largest per-channel
    |beta| + |gamma| / sqrt(var + eps) * sqrt(var) ~ |beta| + |gamma|, scaled to ~2^target"""
    out = {}
    for name, p in wd.items():
        if not name.endswith("_bn"):
            continue
        m = float(np.max(np.abs(p["beta"]) + np.abs(p["gamma"])))
        out[name[:-3]] = int(round(target - np.log2(max(m, 1e-30))))
    return out


def forward(wd, mel, video, qa, qw, sig, stats=None):
    """keras_ref.forward with storage rounding: qa(x, sigma) on every materialised activation, qw on kernels."""
    def store(name, x):
        s = sig.get(name, 0)
        if stats is not None:
            y = (x * 2.0 ** s).abs()
            stats[name] = (float(x.pow(2).mean().sqrt()), float(x.abs().max()),
                           float((y < 2.0 ** -3).to(F64).mean()), s)
        return qa(x, s)

    def conv(x, name, s):
        p = wd[name]
        return K.conv_same(x, qw(p["kernel"], 3), p["bias"], s, F64)

    def deconv(x, name, s):
        p = wd[name]
        return K.deconv_same(x, qw(p["kernel"], 2), p["bias"], s, F64)

    with torch.no_grad():
        a = qa(torch.as_tensor(mel, dtype=F64)[:, None])
        v = qa(torch.as_tensor(video, dtype=F64).permute(0, 3, 1, 2))
        for name, kind, f, k, s, has_bn, pool, _ in K.AUDIO_ENCODER:
            a = K.lrelu(K.bn(conv(a, name, s), wd[name + "_bn"], F64))
            a = store(name if name != "a_conv5" else "concat_a", a)
        for name, kind, f, k, s, has_bn, pool, _ in K.VIDEO_ENCODER:
            v = F.max_pool2d(K.lrelu(K.bn(conv(v, name, s), wd[name + "_bn"], F64)), 2, 2)
            v = store(name if name != "v_conv6" else "concat_v", v)
        N = a.shape[0]
        C, H, W = a.shape[1:]
        x = torch.cat([a.permute(0, 2, 3, 1).reshape(N, -1), v.permute(0, 2, 3, 1).reshape(N, -1)], dim=1)
        for name in ("enc_dense", "dec_dense1"):
            p = wd[name]
            x = K.lrelu(K.bn(x @ torch.as_tensor(qw(p["kernel"], 1), dtype=F64) + torch.as_tensor(p["bias"], dtype=F64),
                             wd[name + "_bn"], F64))
            x = store(name, x)
        p = wd["dec_dense2"]
        x = (x @ torch.as_tensor(qw(p["kernel"], 1), dtype=F64) + torch.as_tensor(p["bias"], dtype=F64)).reshape(N, H, W, C)
        x = store("dec_dense2", K.lrelu(K.bn(x, wd["dec_dense2_bn"], F64, channel_dim=3)).permute(0, 3, 1, 2))
        for name, kind, f, k, s, has_bn, pool, _ in K.AUDIO_DECODER:
            x = deconv(x, name, s)
            if has_bn:
                x = K.lrelu(K.bn(x, wd[name + "_bn"], F64))
                if name != "d_deconv5":          # d_deconv5 feeds the fused d_deconv6 dot in fp32
                    x = store(name, x)
        return x[:, 0].numpy()


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 37
    db = (sys.argv[3] if len(sys.argv) > 3 else "db") == "db"
    torch.set_num_threads(8)
    model = KerasModel.init(seed=seed, randomize=True)
    if db:
        k = model.tensors["d_deconv6/kernel"]
        model.tensors["d_deconv6/kernel"] = (k * 150.0).astype(np.float32)
        model.tensors["d_deconv6/bias"] = np.full_like(model.tensors["d_deconv6/bias"], -40.0)
    rng = np.random.default_rng(seed + 100)
    x = synth_audio(rng, N, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, 640, 160)[0][:, :20] for i in range(N)]).astype(np.float32)
    video = synth_video(rng, N)
    wd = model.layer_dict()
    ref = K.forward(wd, mel, video)
    rms = float(np.sqrt(np.mean(ref ** 2)))
    sig = act_exponents(wd)
    sig["concat_a"] = sig["concat_v"] = min(sig.pop("a_conv5"), sig.pop("v_conv6"))
    stats = {}
    ident = lambda w, ax: w  # noqa: E731
    runs = [("fp32", q_fp32, lambda w, ax: np.asarray(w, np.float32), {}),
            ("pair", q_pair, q_w_pair, {}),
            ("pair+sigma", q_pair, q_w_pair, sig),
            ("pair act only", q_pair, ident, {}),
            ("pair+sigma act only", q_pair, ident, sig)]
    print(f"N={N} seed={seed} db={db} output rms {rms:.4g}")
    for name, qa, qw, sg in runs:
        st = {} if name == "pair" else None
        got = forward(wd, mel, video, qa, qw, sg, st)
        e = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"{name:22s} abs rms {e:.3e}  rel {e / rms:.2e}", flush=True)
        if st:
            stats = st
    print("layer        rms        max      frac(lo subnormal, sigma=0)  sigma(BN rule)")
    for k, (r, m, f, _) in stats.items():
        print(f"{k:12s} {r:9.3g} {m:9.3g}   {f:6.3f}   {sig.get(k, 0)}")


if __name__ == "__main__":
    main()
