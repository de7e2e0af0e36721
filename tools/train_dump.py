"""Debug aid: one grads-only training step on the GPU (N=4, seeded like tests/test_gpu_train.py), the gradients
(minus the three large dense kernels) saved to gpurun_out/train_grads.npz for comparison with the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402

rate = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
dev = torch.device("cuda", 0)
model = KerasModel.init(seed=21, randomize=True)
rng = np.random.default_rng(9)
N = 4
mel = rng.normal(-40, 12, (N, 80, 20)).astype(np.float32)
video = rng.normal(0, 1, (N, 128, 128, 5)).astype(np.float32)
target = (mel + rng.normal(0, 3, mel.shape)).astype(np.float32)
tr = ops.Trainer(model, max_batch=8, device=dev)
loss = tr.step(*[torch.from_numpy(a).to(dev) for a in (mel, video, target)], dropout=rate, seed=1234, grads_only=True)
g = tr.gradients()
skip = ("enc_dense/kernel", "dec_dense1/kernel", "dec_dense2/kernel")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
prm = tr.model().tensors
np.savez(os.path.join(ROOT, "gpurun_out", "train_grads.npz"), loss=float(loss.item()),
         **{k.replace("/", "__"): v for k, v in g.items() if k not in skip},
         **{"P_" + k.replace("/", "__"): v for k, v in prm.items() if k.endswith(("moving_mean", "moving_variance"))})
print("loss", float(loss.item()))
