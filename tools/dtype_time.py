"""Per-stage forward time (HIP events, avse_forward_profile) and whole-step time of the bench workload (B = 512 clips,
STFT + forward) for each compute dtype given on the command line.
    python tools/dtype_time.py [B] [dtype ...]       (default: 512 float32 float32_split bf16)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
import bench  # noqa: E402
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dtypes = sys.argv[2:] or ["float32", "float32_split", "bf16"]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1234)
    a, v = bench.synth(rng, B)
    audio, video = torch.from_numpy(a).to(dev), torch.from_numpy(v).to(dev)
    mean = torch.from_numpy(v.mean(axis=(0, 3)).astype(np.float32)).to(dev)
    std = torch.from_numpy(v.std(axis=(0, 3)).astype(np.float32)).to(dev)
    model = KerasModel.init(seed=0, randomize=True)
    mel = torch.empty((B, 1, 80, 20), dtype=torch.float32, device=dev)
    out = torch.empty((B, 80, 20), dtype=torch.float32, device=dev)
    for dt in dtypes:
        dw = ops.DeviceWeights(model, dt, dev)
        dw.ctx.reserve_for(dw, B)

        def step():
            ops.spectrogram(audio, frames_per_slice=20, out=mel)
            ops.forward(dw, mel.view(B, 80, 20), video, mean, std, out=out, checked=False)
        for _ in range(3):
            step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        _, st = ops.forward_profile(dw, mel.view(B, 80, 20), video, mean, std, out=out)
        top = {k: round(x, 4) for k, x in st.items() if x > 0.01}
        print(f"{dt:14s} step {ms:8.3f} ms = {B / ms * 1e3:10.1f} clips/s; stages {top}", flush=True)
        del dw


if __name__ == "__main__":
    main()
