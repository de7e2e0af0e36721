"""CPU emulation: would Winograd F(2x2, 3x3) keep the split dtype inside the north star's 1e-4 bound?  (VERDICT r5
item 3: "probe fewer products ... on the CPU emulation first".)

The float64 oracle forward (oracle/keras_ref.py semantics, pair-rounded storage of every activation as in
tools/pair_err.py) with the video convolutions computed in float32 arithmetic on pair-rounded operands, either

    direct   F.conv2d in float32 (pair-rounded inputs and per-output-channel scaled pair weights), or
    wino     F(2x2, 3x3): V = B^T d B in float32 from the pair-rounded input tile, V rounded to a pair; U = G g G^T in
             float64, rounded to a per-output-channel scaled pair; M = sum_ci U V in float32; Y = A^T M A in float32.
             5x5 layers (v_conv2) as four 3x3 sub-kernels of the zero-padded 6x6 kernel (offsets 0 / 3 per axis),
             summed in float32 (64 products per 2x2 outputs instead of 100).

and the dB-scale output's absolute RMS error against the float64 forward is printed per scheme.  Products are exact
and sums are float32 in both, so the difference between the lines is what the transforms cost.

    python tools/wino_err.py [N] [seed]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pair_err import K, R, KerasModel, q_pair, q_w_pair, synth_audio, synth_video, act_exponents  # noqa: E402

F64, F32 = torch.float64, torch.float32
BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=F64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=F64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=F64)


def qw_scaled(w, axis_out=0):
    return torch.as_tensor(q_w_pair(w.numpy(), axis_out), dtype=F64)


def wino_sub(xp, g3, oy, ox, H, W):
    """out[y, x] = sum_{a,b<3} xp[y + oy + a, x + ox + b] g3[a, b] over the H x W output grid, by F(2x2, 3x3)."""
    d = xp[:, :, oy:oy + H + 2, ox:ox + W + 2].to(F32)
    d = d.unfold(2, 4, 2).unfold(3, 4, 2)                                     # [N, C, H/2, W/2, 4, 4]
    bt = BT.to(F32)
    V = torch.einsum("ij,nctsjk,lk->nctsil", bt, d, bt)                       # float32 transform
    V = q_pair(V.to(F64)).to(F32)                                              # stored as a pair
    U = torch.einsum("ij,ocjk,lk->ocil", G, g3, G)                            # float64 on the host
    U = qw_scaled(U, 0).to(F32)
    M = torch.einsum("nctsij,ocij->notsij", V, U)                             # float32 sums over ci
    at = AT.to(F32)
    Y = torch.einsum("ij,notsjk,lk->notsil", at, M, at)                       # [N, Co, H/2, W/2, 2, 2]
    N, Co = Y.shape[:2]
    return Y.permute(0, 1, 2, 4, 3, 5).reshape(N, Co, H, W)


def f32(t):
    return t.to(F32).to(F64)


def mfma_direct(x, g, pad):
    """The stream kernels' arithmetic: K in blocks of (16 channels x 1 tap), each block's products summed exactly and
    added to the float32 accumulator with one rounding (v_mfma_f32_16x16x32_f16: 32 exact products, one rounding;
    DESIGN.md §3 split-f16 'Numerics on the hardware'), blocks in chunk-major, tap-minor order."""
    Co, Ci, k, _ = g.shape
    N, C, H, W = x.shape
    xp = F.pad(x, (pad, pad, pad, pad))
    gq = qw_scaled(g, 0)
    acc = torch.zeros(N, Co, H, W, dtype=F64)
    for c0 in range(0, Ci, 16):
        for ky in range(k):
            for kx in range(k):
                xs = xp[:, c0:c0 + 16, ky:ky + H, kx:kx + W]
                part = torch.einsum("nchw,oc->nohw", xs, gq[:, c0:c0 + 16, ky, kx])
                acc = f32(acc + part)
    return acc


def mfma_wino_sub(xp, g3, oy, ox, H, W):
    """wino_sub with the MFMA accumulation model: M = sum over ci blocks of 16 (exact within a block, one float32
    rounding per block); the transforms in float32 with a rounding per operation."""
    d = xp[:, :, oy:oy + H + 2, ox:ox + W + 2]
    d = d.unfold(2, 4, 2).unfold(3, 4, 2)                                     # [N, C, H/2, W/2, 4, 4]
    t = torch.stack([f32(d[..., 0, :] - d[..., 2, :]), f32(d[..., 1, :] + d[..., 2, :]),
                     f32(d[..., 2, :] - d[..., 1, :]), f32(d[..., 1, :] - d[..., 3, :])], dim=-2)
    V = torch.stack([f32(t[..., 0] - t[..., 2]), f32(t[..., 1] + t[..., 2]),
                     f32(t[..., 2] - t[..., 1]), f32(t[..., 1] - t[..., 3])], dim=-1)
    V = q_pair(V)
    U = qw_scaled(torch.einsum("ij,ocjk,lk->ocil", G, g3, G), 0)
    N, Ci = V.shape[:2]
    Co = U.shape[0]
    M = torch.zeros(N, Co, H // 2, W // 2, 4, 4, dtype=F64)
    for c0 in range(0, Ci, 16):
        M = f32(M + torch.einsum("nctsij,ocij->notsij", V[:, c0:c0 + 16], U[:, c0:c0 + 16]))
    r = torch.stack([f32(f32(M[..., 0, :] + M[..., 1, :]) + M[..., 2, :]),
                     f32(f32(M[..., 1, :] - M[..., 2, :]) - M[..., 3, :])], dim=-2)      # A^T M
    Y = torch.stack([f32(f32(r[..., 0] + r[..., 1]) + r[..., 2]),
                     f32(f32(r[..., 1] - r[..., 2]) - r[..., 3])], dim=-1)               # (A^T M) A
    return Y.permute(0, 1, 2, 4, 3, 5).reshape(N, Co, H, W)


def conv_video(x, p, mode):
    """'same' stride-1 conv of network.py:139-169 in float32 arithmetic; x float64 (already pair-rounded)."""
    g = torch.as_tensor(np.asarray(p["kernel"], np.float32), dtype=F64).permute(3, 2, 0, 1)   # [Co, Ci, k, k]
    k = g.shape[-1]
    N, C, H, W = x.shape
    bias = torch.as_tensor(np.asarray(p["bias"], np.float32), dtype=F32)
    if mode == "mfma":
        return mfma_direct(x, g, k // 2) + bias.to(F64)[None, :, None, None]
    if mode == "mfma_wino":
        if k == 3:
            y = mfma_wino_sub(F.pad(x, (1, 1, 1, 1)), g, 0, 0, H, W)
        else:
            g6 = torch.zeros(g.shape[0], g.shape[1], 6, 6, dtype=F64)
            g6[:, :, :5, :5] = g
            xp = F.pad(x, (2, 3, 2, 3))
            y = None
            for oy in (0, 3):
                for ox in (0, 3):
                    part = mfma_wino_sub(xp, g6[:, :, oy:oy + 3, ox:ox + 3], oy, ox, H, W)
                    y = part if y is None else f32(y + part)
        return y + bias.to(F64)[None, :, None, None]
    if mode == "direct":
        # Keras 'same' padding for odd k: symmetric k // 2
        y = F.conv2d(x.to(F32), qw_scaled(g, 0).to(F32), None, 1, k // 2)
    elif k == 3:
        y = wino_sub(F.pad(x, (1, 1, 1, 1)), g, 0, 0, H, W)
    else:
        g6 = torch.zeros(g.shape[0], g.shape[1], 6, 6, dtype=F64)
        g6[:, :, :5, :5] = g
        xp = F.pad(x, (2, 3, 2, 3))
        y = None
        for oy in (0, 3):
            for ox in (0, 3):
                part = wino_sub(xp, g6[:, :, oy:oy + 3, ox:ox + 3], oy, ox, H, W)
                y = part if y is None else y + part
    return (y + bias[None, :, None, None]).to(F64)


def forward(wd, mel, video, modes, sig):
    """pair_err.forward with the video convolutions of `modes` ({layer: 'direct' | 'wino'}) in float32 arithmetic."""
    with torch.no_grad():
        a = q_pair(torch.as_tensor(mel, dtype=F64)[:, None])
        v = q_pair(torch.as_tensor(video, dtype=F64).permute(0, 3, 1, 2))
        for name, kind, f, k, s, has_bn, pool, _ in K.AUDIO_ENCODER:
            p = wd[name]
            a = K.lrelu(K.bn(K.conv_same(a, q_w_pair(p["kernel"], 3), p["bias"], s, F64), wd[name + "_bn"], F64))
            a = q_pair(a, sig.get(name, 0))
        for name, kind, f, k, s, has_bn, pool, _ in K.VIDEO_ENCODER:
            p = wd[name]
            if name in modes:
                z = conv_video(v, p, modes[name])
            else:
                z = K.conv_same(v, q_w_pair(p["kernel"], 3), p["bias"], s, F64)
            v = F.max_pool2d(K.lrelu(K.bn(z, wd[name + "_bn"], F64)), 2, 2)
            v = q_pair(v, sig.get(name, 0))
        N = a.shape[0]
        C, H, W = a.shape[1:]
        x = torch.cat([a.permute(0, 2, 3, 1).reshape(N, -1), v.permute(0, 2, 3, 1).reshape(N, -1)], dim=1)
        for name in ("enc_dense", "dec_dense1"):
            p = wd[name]
            x = K.lrelu(K.bn(x @ torch.as_tensor(q_w_pair(p["kernel"], 1), dtype=F64)
                             + torch.as_tensor(p["bias"], dtype=F64), wd[name + "_bn"], F64))
            x = q_pair(x)
        p = wd["dec_dense2"]
        x = (x @ torch.as_tensor(q_w_pair(p["kernel"], 1), dtype=F64)
             + torch.as_tensor(p["bias"], dtype=F64)).reshape(N, H, W, C)
        x = q_pair(K.lrelu(K.bn(x, wd["dec_dense2_bn"], F64, channel_dim=3)).permute(0, 3, 1, 2))
        for name, kind, f, k, s, has_bn, pool, _ in K.AUDIO_DECODER:
            p = wd[name]
            x = K.deconv_same(x, q_w_pair(p["kernel"], 2), p["bias"], s, F64)
            if has_bn:
                x = K.lrelu(K.bn(x, wd[name + "_bn"], F64))
                if name != "d_deconv5":
                    x = q_pair(x)
        return x[:, 0].numpy()


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 37
    torch.set_num_threads(8)
    model = KerasModel.init(seed=seed, randomize=True)
    k = model.tensors["d_deconv6/kernel"]
    model.tensors["d_deconv6/kernel"] = (k * 150.0).astype(np.float32)          # dB-scale output (pair_err.py)
    model.tensors["d_deconv6/bias"] = np.full_like(model.tensors["d_deconv6/bias"], -40.0)
    rng = np.random.default_rng(seed + 100)
    x = synth_audio(rng, N, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, 640, 160)[0][:, :20] for i in range(N)]).astype(np.float32)
    video = synth_video(rng, N)
    wd = model.layer_dict()
    ref = K.forward(wd, mel, video)
    rms = float(np.sqrt(np.mean(ref ** 2)))
    print(f"N={N} seed={seed} dB-scale output rms {rms:.4g}")
    vids = ["v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5", "v_conv6"]
    mf = {n: "mfma" for n in vids[1:5]}
    schemes = [("MFMA-block sums, v_conv2..5 direct", mf),
               ("MFMA-block sums, wino v_conv3..5", {**mf, **{n: "mfma_wino" for n in vids[2:5]}}),
               ("MFMA-block sums, wino v_conv2..5", {**mf, **{n: "mfma_wino" for n in vids[1:5]}})]
    for name, modes in schemes:
        got = forward(wd, mel, video, modes, {})
        e = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"{name:42s} abs rms {e:.3e}  rel {e / rms:.2e}", flush=True)
    if os.environ.get("WINO_ALL") is None:
        return
    schemes = [("pair storage, video convs float64 sums", {}),
               ("direct float32 sums, every video conv", {n: "direct" for n in vids[1:]}),
               ("wino F(2,3) on v_conv3..5", {**{n: "direct" for n in vids[1:]}, **{n: "wino" for n in vids[2:5]}}),
               ("wino on v_conv3..6", {**{n: "direct" for n in vids[1:]}, **{n: "wino" for n in vids[2:6]}}),
               ("wino v_conv2 (4 x F(2,3)) + v_conv3..5", {**{n: "direct" for n in vids[1:]},
                                                          **{n: "wino" for n in vids[1:5]}})]
    for name, modes in schemes:
        got = forward(wd, mel, video, modes, {})
        e = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"{name:42s} abs rms {e:.3e}  rel {e / rms:.2e}", flush=True)


if __name__ == "__main__":
    main()
