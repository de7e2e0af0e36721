"""Run the bf16 forward (and the spectrogram) a few times at the bench shape — a target for
rocprofv3 kernel traces / PMC passes (tools/profile.sh)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402


def main():
    B = int(os.environ.get("AVSE_B", "512"))
    reps = int(os.environ.get("AVSE_REPS", "5"))
    dtype = os.environ.get("AVSE_DTYPE", "bf16")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    audio = torch.from_numpy(rng.normal(0, 3000, (B, 3200)).astype(np.float32)).to(dev)
    video = torch.from_numpy(rng.integers(0, 256, (B, 128, 128, 5)).astype(np.float32)).to(dev)
    mean = video.mean(dim=(0, 3)).contiguous()
    std = video.std(dim=(0, 3)).contiguous()
    dw = ops.DeviceWeights(KerasModel.init(seed=0, randomize=True), dtype)
    out = torch.empty((B, 80, 20), device=dev)
    for _ in range(reps):
        mel = ops.spectrogram(audio, frames_per_slice=20)
        ops.forward(dw, mel.view(B, 80, 20), video, mean, std, out=out)
    torch.cuda.synchronize()
    print("done", float(out.float().abs().mean()))


if __name__ == "__main__":
    main()
