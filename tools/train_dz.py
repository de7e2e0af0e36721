"""Debug aid: dL/dz of one BN layer (AVSE_TRAIN_DEBUG_STOP) after a grads-only step, saved to gpurun_out/dz_<layer>.npy."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import _lib, ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402

layer = int(sys.argv[1])
mode = int(sys.argv[4]) if len(sys.argv) > 4 else 2   # 2: dz after the BN backward, 4: dL/d(input)
count = int(sys.argv[2])
rate = float(sys.argv[3]) if len(sys.argv) > 3 else 0.25
dev = torch.device("cuda", 0)
model = KerasModel.init(seed=21, randomize=True)
rng = np.random.default_rng(9)
N = 4
mel = rng.normal(-40, 12, (N, 80, 20)).astype(np.float32)
video = rng.normal(0, 1, (N, 128, 128, 5)).astype(np.float32)
target = (mel + rng.normal(0, 3, mel.shape)).astype(np.float32)
tr = ops.Trainer(model, max_batch=8, device=dev)
a, v, t = [torch.from_numpy(x).to(dev) for x in (mel, video, target)]
loss = torch.zeros((), dtype=torch.float32, device=dev)
_lib.check(_lib.load().avse_trainer_step(tr.handle, _lib.ptr(a), _lib.ptr(v), _lib.ptr(t), None, None, N, 5e-4, rate, 1234,
                                         1 | mode | (layer << 8), _lib.ptr(loss), _lib.stream_handle(dev)), "step")
out = np.empty(count, np.float32)
_lib.check(_lib.load().avse_trainer_read(tr.handle, 4, out.ctypes.data_as(ctypes.c_void_p), count), "read")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"dz_{layer}_{rate}_{mode}.npy"), out)
print("saved", count)
