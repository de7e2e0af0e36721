"""Per-phase cycles of k_istft_fused (istft.hip) at the configs[4] ISTFT (667 x 3-s utterances), from a diagnostic
variant library built with -DAVSE_ISTFT_STAMP (s_memtime stamps of thread 0 per block, summed over items):
    make -C audio-visual-speech-enhancement_amd/csrc_ab OUT=$PWD/tools/_libavse_stamp.so EXTRA=-DAVSE_ISTFT_STAMP
    python tools/istft_stamps.py tools/_libavse_stamp.so"""
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
from avse_amd import _lib, ops  # noqa: E402

PHASES = ["1 amplitudes", "2 Gram MFMA solve", "3 spectrum x phase", "4a Z' -> regs", "4b dft20 -> LDS", "4c -> regs",
          "4d dft16 -> LDS", "5b overlap-add", "5a next item's loads"]


def main():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    U = 667
    t = np.arange(48000) / 16000.0
    utt = (rng.normal(0, 3000, (U, 48000)) + 3000 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    utt = torch.from_numpy(utt).to(dev)
    mel, stft = ops.spectrogram(utt, frames_per_slice=20, return_stft=True)
    lib = _lib.load()
    fn = lib.avse_istft_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((1024, 9), dtype=np.uint64)
    for _ in range(3):
        ops.istft(mel, stft)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    reps = 5
    for _ in range(reps):
        ops.istft(mel, stft)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, 1)
    OF = int(os.environ.get("AVSE_ISTFT_OF", "30"))   # output hops per chunk of the library measured
    items = U * ((300 - 1 + OF - 1) // OF) * reps
    tot = buf[:, :9].sum(axis=0).astype(np.float64)
    print(f"cycles per item (thread 0 of each block, {items} items):")
    for name, v in zip(PHASES, tot):
        print(f"  {name:22s} {v / items:9.0f}")
    print(f"  {'total':22s} {tot.sum() / items:9.0f}")


if __name__ == "__main__":
    main()
