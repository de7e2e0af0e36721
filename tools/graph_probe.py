"""Whole-step timing: direct launches vs the same step captured in a torch CUDA(HIP) graph (bench.py's workload).
Measures the inter-kernel idle time a graph removes.   python tools/graph_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402
from bench import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 512
    model = KerasModel.init(seed=0, randomize=True)
    dw = ops.DeviceWeights(model, "bf16", dev)
    dw.ctx.reserve(B, dw.dtype)
    audio_np, video_np = synth(np.random.default_rng(1234), B)
    audio, video = torch.from_numpy(audio_np).to(dev), torch.from_numpy(video_np).to(dev)
    mean = torch.from_numpy(video_np.mean(axis=(0, 3)).astype(np.float32)).to(dev)
    std = torch.from_numpy(video_np.std(axis=(0, 3)).astype(np.float32)).to(dev)
    out = torch.empty((B, 80, 20), dtype=torch.float32, device=dev)
    mel = torch.empty((B, 1, 80, 20), dtype=torch.float32, device=dev)

    def step():
        m = ops.spectrogram(audio, frames_per_slice=20)
        ops.forward(dw, m.view(B, 80, 20), video, mean, std, out=out)

    def timed(fn, n=20):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    ref = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    diff = (out - ref).abs().max().item()
    print(f"direct {timed(step):.4f} ms/step   graph {timed(g.replay):.4f} ms/step   max|graph - direct| {diff:.3g}",
          flush=True)


if __name__ == "__main__":
    main()
