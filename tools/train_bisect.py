"""Bisect the batch size at which the trainer's gradients leave the N = 3 result (tests/test_gpu_train.py
test_max_batch_1023_equals_repeated_small_batch): a 3-clip batch repeated k times has the N = 3 gradients exactly.
GPU box:  python tools/train_bisect.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402
from test_gpu_train import batch, rel_rms  # noqa: E402

WATCH = ["d_deconv6/kernel", "d_deconv5_bn/gamma", "d_deconv5/kernel", "d_deconv4_bn/beta", "d_deconv4/kernel",
         "enc_dense/kernel", "a_conv1/kernel"]


def grads(model, arrays, max_batch, gpu):
    tr = ops.Trainer(model, max_batch=max_batch, device=gpu)
    loss = float(tr.step(*[torch.from_numpy(a).to(gpu) for a in arrays], dropout=0.0, grads_only=True).item())
    g = tr.gradients()
    del tr
    torch.cuda.empty_cache()
    return loss, g


def main():
    gpu = torch.device("cuda", 0)
    model = KerasModel.init(seed=23, randomize=True)
    small = batch(np.random.default_rng(31), 3)
    l3, g3 = grads(model, small, 3, gpu)
    ks = [int(x) for x in sys.argv[1:]] or [1, 2, 8, 32, 100, 200, 341]
    for k in ks:
        rep = [np.ascontiguousarray(np.tile(a, (k,) + (1,) * (a.ndim - 1))) for a in small]
        for mb in sorted({3 * k, 1023}):
            if mb < 3 * k:
                continue
            l, g = grads(model, rep, mb, gpu)
            errs = " ".join(f"{n.split('/')[0][:10]}:{rel_rms(g[n], g3[n]):.1e}" for n in WATCH)
            print(f"k={k:4d} N={3 * k:5d} max_batch={mb:5d} loss rel {abs(l - l3) / abs(l3):.1e}  {errs}", flush=True)


if __name__ == "__main__":
    main()
