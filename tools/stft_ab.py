"""K1 A/B on the GPU box: time the configs[1] STFT leg with a variant library and dump its outputs for comparison.
  python tools/stft_ab.py run LIB TAG     -> prints the leg timing, saves gpurun_out/stft_ab_TAG.npz
  python tools/stft_ab.py cmp TAG_A TAG_B -> max / rms |dB| differences of every saved output
Outputs: the bench batch (4096 x 3200, 20-frame slices), plain [80, 21] layout, 40 mel bands, zero padding,
top_db off, and an odd batch (B = 7: fewer blocks than the persistent grid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def run(lib, tag):
    import torch
    sys.path.insert(0, ROOT)
    import avse_pkg
    avse_pkg.load()
    sys.modules["avse_amd"]._lib.LIB_PATH = os.path.abspath(lib)
    import bench
    from avse_amd import ops
    dev = torch.device("cuda", 0)
    print(tag, "configs[1] leg:", bench.leg_stft(dev), flush=True)
    rng = np.random.default_rng(7)
    sig = torch.from_numpy(bench.synth(rng, 4096, video=False)[0]).to(dev)
    res = {
        "seg": ops.spectrogram(sig, frames_per_slice=20)[::8],
        "plain": ops.spectrogram(sig[:300]),
        "mel40": ops.spectrogram(sig[:300], n_mels=40, frames_per_slice=20),
        "zero": ops.spectrogram(sig[:300], pad_mode="constant", frames_per_slice=20),
        "notop": ops.spectrogram(sig[:300], top_db=None),
        "odd": ops.spectrogram(sig[:7], frames_per_slice=20),
    }
    torch.cuda.synchronize()
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"stft_ab_{tag}.npz"), **{k: v.cpu().numpy() for k, v in res.items()})


def cmp(ta, tb):
    a = np.load(os.path.join(OUT, f"stft_ab_{ta}.npz"))
    b = np.load(os.path.join(OUT, f"stft_ab_{tb}.npz"))
    worst = 0.0
    for k in a.files:
        d = np.abs(a[k].astype(np.float64) - b[k])
        worst = max(worst, float(d.max()))
        print(f"{ta} vs {tb} {k:6s} shape {a[k].shape}: max {d.max():.3e} dB  rms {np.sqrt((d ** 2).mean()):.3e} dB")
    print("worst", worst)
    return 0 if worst <= 1e-3 else 1


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
