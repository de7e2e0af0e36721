"""STFT / ISTFT timing on the GPU box: configs[1] leg (B = 4096 segments, rotated buffers), the B = 512 bench
batch, and the configs[4] utterance batch (667 x 48000 samples with the complex STFT kept) + its ISTFT.
Kernel times come from HIP events around `reps` back-to-back launches (python launch overhead included;
rocprofv3 --kernel-trace gives the kernel-only figure)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
if len(sys.argv) > 1:                       # A/B: a variant library built with make OUT=... BUILD=... EXTRA=...
    sys.modules["avse_amd"]._lib.LIB_PATH = os.path.abspath(sys.argv[1])
    print("library:", sys.argv[1])
import bench  # noqa: E402
from avse_amd import ops  # noqa: E402


def timed(fn, reps):
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
    dev = torch.device("cuda", 0)
    print("configs[1] leg:", bench.leg_stft(dev))
    rng = np.random.default_rng(0)
    seg = torch.from_numpy(bench.synth(rng, 512, video=False)[0]).to(dev)
    out = torch.empty((512, 1, 80, 20), dtype=torch.float32, device=dev)
    print("B=512 segments: %.4f ms" % timed(lambda: ops.spectrogram(seg, frames_per_slice=20, out=out), 50))
    U = 667
    t = np.arange(48000) / 16000.0
    utt = (rng.normal(0, 3000, (U, 48000)) + 3000 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    utt = torch.from_numpy(utt).to(dev)
    box = {}

    def spec():
        box["mel"], box["stft"] = ops.spectrogram(utt, frames_per_slice=20, return_stft=True)

    print("e2e STFT (667 x 48000, complex kept): %.4f ms" % timed(spec, 10))
    mel = box["mel"]
    stft = box["stft"]
    print("e2e ISTFT: %.4f ms" % timed(lambda: ops.istft(mel, stft), 10))


if __name__ == "__main__":
    main()
