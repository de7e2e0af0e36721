"""Per-step cycles of k_spec_seg / k_spec640 (stft.hip) on BASELINE configs[1] (4096 segments, no complex STFT output), from a
diagnostic variant library built with -DAVSE_STFT_STAMP (s_memtime stamps of thread 0 of every block):
    make -C audio-visual-speech-enhancement_amd/csrc_ab OUT=$PWD/tools/_libavse_sstamp.so EXTRA=-DAVSE_STFT_STAMP
    python tools/stft_stamps.py tools/_libavse_sstamp.so
k_spec_seg (the configs[1] kernel since r03e) loops over utterances: the figures are per utterance.  k_spec640 runs
for other geometries; its step names apply when the second argument is 640 (forced with -DAVSE_NO_SEG)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
sys.modules["avse_amd"]._lib.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
from avse_amd import _lib, ops  # noqa: E402

STEPS = ["0 samples issue + barrier", "1 dft20 (wave 0)", "2a -> regs", "2b dft16", "3 untangle + |X|", "4 mel + dB + max",
         "5 clamp + store"]
STEPS_SEG = ["0 DMA wait", "1 dft20 + twiddle", "2 dft16", "3 untangle + |X|", "4 mel + dB + DMA + barrier", "5 dB stores"]
if len(sys.argv) < 3 or sys.argv[2] != "640":
    STEPS = STEPS_SEG


def main():
    dev = torch.device("cuda", 0)
    B = 4096
    seg = torch.from_numpy(bench.synth(np.random.default_rng(0), B, video=False)[0]).to(dev)
    out = torch.empty((B, 1, 80, 20), dtype=torch.float32, device=dev)
    fn = _lib.load().avse_spec_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((4096, 8), dtype=np.uint64)
    for _ in range(3):
        ops.spectrogram(seg, frames_per_slice=20, out=out)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    reps = 10
    for _ in range(reps):
        ops.spectrogram(seg, frames_per_slice=20, out=out)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    blocks = B * reps
    print(f"cycles per utterance (thread 0 of its block, {blocks} 21-frame segments):")
    tot = buf.sum(axis=0).astype(np.float64)
    for name, v in zip(STEPS + [""] * (8 - len(STEPS)), tot):
        if not name:
            continue
        print(f"  {name:22s} {v / blocks:9.0f}")
    print(f"  {'total':22s} {tot.sum() / blocks:9.0f}")


if __name__ == "__main__":
    main()
