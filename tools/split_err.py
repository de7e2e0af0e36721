"""CPU emulation: output error of fp32-accurate split-bf16 arithmetic schemes for the video convolutions, against
the float64 oracle, next to the plain-fp32 scheme — which scheme can carry the north star's 1e-4 absolute RMS bound
on dB-scale outputs (DESIGN.md §3 "split-bf16").  Every conv is evaluated in float64 over the products the scheme
keeps (products of bf16 pieces are exact in float64), its output rounded to float32 like an fp32 accumulator + fp32
epilogue; so the differences between schemes are representation / dropped-product errors, not accumulation order.

    python tools/split_err.py [N] [seed]
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


def split(t, n, dt=torch.bfloat16):
    """t (float64 holding float32 values) -> n pieces of dtype dt, t ~= sum(pieces) (each piece rounds the residual)."""
    out, r = [], t
    for _ in range(n):
        p = r.to(dt).to(torch.float64)
        out.append(p)
        r = r - p
    return out


SCHEMES = {
    # name: (pieces of x, pieces of w, kept (i, j) products)
    "fp32": None,
    "bf16x9": (3, 3, [(i, j) for i in range(3) for j in range(3)]),
    "bf16x6": (3, 3, [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0)]),
    "bf16x5-nomm": (3, 3, [(0, 0), (0, 1), (1, 0), (0, 2), (2, 0)]),
    "bf16x5-a2": (2, 3, [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2)]),
    "bf16x4-a2": (2, 3, [(0, 0), (0, 1), (1, 0), (0, 2)]),
    "bf16x3": (2, 2, [(0, 0), (0, 1), (1, 0)]),
    "fp16x3": (2, 2, [(0, 0), (0, 1), (1, 0)], torch.float16, True),
    "fp16x3-noscale": (2, 2, [(0, 0), (0, 1), (1, 0)], torch.float16, False),
    "fp16x4": (2, 2, [(0, 0), (0, 1), (1, 0), (1, 1)], torch.float16, True),
}


def make_conv(scheme, layers):
    orig = K.conv_same

    def conv(x, kernel, bias, strides, dtype):
        kh, kw, cin, cout = kernel.shape
        is_video = x.shape[2] >= 4 and x.shape[2] == x.shape[3] and x.shape[2] in (128, 64, 32, 16, 8, 4)
        name = {128: "v_conv1", 64: "v_conv2", 32: "v_conv3", 16: "v_conv4", 8: "v_conv5", 4: "v_conv6"}.get(x.shape[2])
        w = torch.as_tensor(np.asarray(kernel, np.float32), dtype=torch.float64)
        if scheme is None or not is_video or name not in layers:
            y = orig(x.to(torch.float32).to(torch.float64), w.numpy(), bias, strides, torch.float64)
        else:
            sch = SCHEMES[scheme]
            na, nb, prods = sch[:3]
            dt = sch[3] if len(sch) > 3 else torch.bfloat16
            wsc = 1.0
            if len(sch) > 4 and sch[4]:
                wsc = 2.0 ** (14 - int(np.ceil(np.log2(float(w.abs().max())))))
            xs = split(x.to(torch.float32).to(torch.float64), na, dt)
            ws = [p / wsc for p in split(w * wsc, nb, dt)]
            y = None
            for i, j in prods:
                t = orig(xs[i], ws[j].numpy(), np.zeros_like(bias), strides, torch.float64)
                y = t if y is None else y + t
            y = y + torch.as_tensor(bias, dtype=torch.float64).view(1, -1, 1, 1)
        return y.to(torch.float32).to(torch.float64)
    return conv


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 37
    torch.set_num_threads(8)
    model = KerasModel.init(seed=seed, randomize=True)
    k = model.tensors["d_deconv6/kernel"]
    model.tensors["d_deconv6/kernel"] = (k * 150.0).astype(np.float32)     # dB-scale output (test_gpu_forward.db_scale)
    model.tensors["d_deconv6/bias"] = np.full_like(model.tensors["d_deconv6/bias"], -40.0)
    rng = np.random.default_rng(seed + 100)
    x = synth_audio(rng, N, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, 640, 160)[0][:, :20] for i in range(N)]).astype(np.float32)
    video = synth_video(rng, N)
    if len(sys.argv) > 3 and sys.argv[3] == "norm":
        m, s = R.video_normalizer_fit(video)
        video = R.video_normalize(video, m, s).astype(np.float32)
    wd = model.layer_dict()
    ref = K.forward(wd, mel, video)
    rms = float(np.sqrt(np.mean(ref ** 2)))
    layers_sets = {"v1-v5": {"v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5"},
                   "v1-v6": {"v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5", "v_conv6"}}
    orig = K.conv_same
    print(f"N={N} seed={seed} output rms {rms:.4g}")
    for sname in SCHEMES:
        for lname, ls in layers_sets.items():
            if sname == "fp32" and lname != "v1-v5":
                continue
            K.conv_same = make_conv(SCHEMES[sname] and sname, ls)
            try:
                got = K.forward(wd, mel, video)
            finally:
                K.conv_same = orig
            e = float(np.sqrt(np.mean((got - ref) ** 2)))
            print(f"{sname:12s} {lname:6s} abs rms {e:.3e}  rel {e / rms:.2e}", flush=True)


if __name__ == "__main__":
    main()
