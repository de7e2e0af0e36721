"""Forward per-stage time (avse_forward_profile) and STFT time at B clips for the three frame-rate networks:
25 fps ([80, 20] x 5 frames), 29.97 fps ([80, 24] x 5) and 30 fps ([80, 24] x 6), in each dtype given.
    python tools/fps_time.py [B] [dtype ...]        (default: 512 float32_split bf16)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import ops  # noqa: E402
from avse_amd.data_processor import frame_geometry  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402

NETS = [(25.0, 20, 5), (29.97, 24, 5), (30.0, 24, 6)]


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dtypes = sys.argv[2:] or ["float32_split", "bf16"]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    for fps, T, F in NETS:
        g = frame_geometry(16000, 200, 1, fps)
        seg = g["samples_per_slice"]
        audio = torch.from_numpy(rng.normal(0, 3000, (B, seg)).astype(np.float32)).to(dev)
        mel = torch.empty((B, 1, 80, T), dtype=torch.float32, device=dev)
        stft_ms = timed(lambda: ops.spectrogram(audio, n_fft=g["n_fft"], hop_length=g["hop_length"],
                                                frames_per_slice=T, out=mel))
        v = rng.integers(0, 256, (B, 128, 128, F)).astype(np.float32)
        video = torch.from_numpy(v).to(dev)
        mean = torch.from_numpy(v.mean(axis=(0, 3)).astype(np.float32)).to(dev)
        std = torch.from_numpy(v.std(axis=(0, 3)).astype(np.float32)).to(dev)
        model = KerasModel.init(seed=0, randomize=True, audio_shape=(80, T), video_shape=(128, 128, F))
        out = torch.empty((B, 80, T), dtype=torch.float32, device=dev)
        # ISTFT (K6) of 64 3-s utterances at this rate: analysis STFT with the complex output, then the inverse
        xu = torch.from_numpy(rng.normal(0, 3000, (64, 48000)).astype(np.float32)).to(dev)
        melu, D = ops.spectrogram(xu, n_fft=g["n_fft"], hop_length=g["hop_length"], frames_per_slice=T,
                                  return_stft=True)
        istft_ms = timed(lambda: ops.istft(melu, D, n_fft=g["n_fft"], hop_length=g["hop_length"]))
        print(f"{fps:5.2f} fps n_fft {g['n_fft']} ISTFT of 64 x 3 s: {istft_ms:.4f} ms", flush=True)
        for dt in dtypes:
            dw = ops.DeviceWeights(model, dt, dev)
            dw.ctx.reserve_for(dw, B)
            ms = timed(lambda: ops.forward(dw, mel.view(B, 80, T), video, mean, std, out=out, checked=False))
            _, st = ops.forward_profile(dw, mel.view(B, 80, T), video, mean, std, out=out)
            top = {k: round(x, 4) for k, x in st.items() if x > 0.01}
            print(f"{fps:5.2f} fps n_fft {g['n_fft']} STFT {stft_ms:.4f} ms | {dt:14s} forward {ms:8.3f} ms "
                  f"({B / (ms + stft_ms) * 1e3:9.1f} clips/s with STFT); stages {top}", flush=True)
            del dw


if __name__ == "__main__":
    main()
