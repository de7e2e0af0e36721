"""A target for rocprofv3 kernel traces / PMC passes (tools/profile.sh): the bench's bf16 forward (+ spectrogram)
at B = 512 a few times, or with AVSE_MODE=stft the configs[1] STFT at B = 4096 over 5 rotated buffer sets."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_pkg  # noqa: E402

avse_pkg.load()
import bench  # noqa: E402
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402


def main():
    mode = os.environ.get("AVSE_MODE", "forward")
    reps = int(os.environ.get("AVSE_REPS", "5"))
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1234)
    if mode == "stft":
        B, sets = 4096, 5
        ins = [torch.from_numpy(bench.synth(rng, B, video=False)[0]).to(dev) for _ in range(sets)]
        for k in range(sets * reps):
            ops.spectrogram(ins[k % sets], frames_per_slice=20)
        torch.cuda.synchronize()
        print("done stft")
        return
    B = int(os.environ.get("AVSE_B", "512"))
    dtype = os.environ.get("AVSE_DTYPE", "bf16")
    audio_np, video_np = bench.synth(rng, B)
    audio, video = torch.from_numpy(audio_np).to(dev), torch.from_numpy(video_np).to(dev)
    mean = torch.from_numpy(video_np.mean(axis=(0, 3)).astype(np.float32)).to(dev)
    std = torch.from_numpy(video_np.std(axis=(0, 3)).astype(np.float32)).to(dev)
    dw = ops.DeviceWeights(KerasModel.init(seed=0, randomize=True), dtype)
    out = torch.empty((B, 80, 20), device=dev)
    for _ in range(reps):
        mel = ops.spectrogram(audio, frames_per_slice=20)
        ops.forward(dw, mel.view(B, 80, 20), video, mean, std, out=out)
    torch.cuda.synchronize()
    print("done", float(out.float().abs().mean()))


if __name__ == "__main__":
    main()
