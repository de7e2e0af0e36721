"""Debug: fused v_conv1 (conv_v1r.hip) vs the generic k_conv path at batch N, per clip and per 16x16 tile."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import avse_pkg  # noqa: F401
import bench
from avse_amd import ops
from avse_amd.model import KerasModel
from test_gpu_forward import scratch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 301
rng = np.random.default_rng(1234)
audio_np, video_np = bench.synth(rng, N)
mean_np = video_np.mean(axis=(0, 3)).astype(np.float32)
std_np = video_np.std(axis=(0, 3)).astype(np.float32)
model = KerasModel.init(seed=0, randomize=True)
mel = torch.zeros((N, 80, 20), device="cuda")
args = [mel, ops.to_device(video_np), ops.to_device(mean_np), ops.to_device(std_np)]
dw = ops.DeviceWeights(model, "bf16")
ops.forward(dw, *args)
clips = list(range(0, N, max(1, N // 40)))
a = scratch(dw, N, clips, ["v_conv1"])["v_conv1"]
with dw.ctx.options(no_halo=1):
    dg = ops.DeviceWeights(model, "bf16")
ops.forward(dg, *args)
b = scratch(dg, N, clips, ["v_conv1"])["v_conv1"]
print("shape", a.shape)
d = np.abs(a - b)
for ci, c in enumerate(clips):
    t = d[ci].reshape(8, 8, 8, 8, -1).max(axis=(1, 3, 4))   # [tile y][tile x] (pooled 64x64 -> 8x8 tiles)
    bad = np.argwhere(t > 0.05 * (np.abs(b[ci]).max() + 1e-6))
    if len(bad):
        print("clip", c, "bad tiles", [tuple(x) for x in bad][:10], "max", t.max())
print("global rel rms", np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(b ** 2)))
