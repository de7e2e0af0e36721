"""Per-stage forward times (HIP events between launches, avse_forward_profile), median of R reps.
    AVSE_B=512 AVSE_DTYPE=bf16 python tools/stage_times.py [label]"""
import json
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
    reps = int(os.environ.get("AVSE_REPS", "7"))
    dtype = os.environ.get("AVSE_DTYPE", "bf16")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    audio = torch.from_numpy(rng.normal(0, 3000, (B, 3200)).astype(np.float32)).to(dev)
    video = torch.from_numpy(rng.integers(0, 256, (B, 128, 128, 5)).astype(np.float32)).to(dev)
    mean = video.mean(dim=(0, 3)).contiguous()
    std = video.std(dim=(0, 3)).contiguous()
    dw = ops.DeviceWeights(KerasModel.init(seed=0, randomize=True), dtype)
    mel = ops.spectrogram(audio, frames_per_slice=20).view(B, 80, 20)
    out = torch.empty((B, 80, 20), device=dev)
    runs = []
    for _ in range(reps + 2):
        _, st = ops.forward_profile(dw, mel, video, mean, std, out=out)
        runs.append(st)
    runs = runs[2:]
    med = {k: float(np.median([r[k] for r in runs])) for k in runs[0]}
    label = sys.argv[1] if len(sys.argv) > 1 else ""
    print(json.dumps({"label": label, "B": B, "dtype": dtype, "total_ms": round(sum(med.values()), 4),
                      "stage_ms": {k: round(v, 4) for k, v in med.items()}}))


if __name__ == "__main__":
    main()
