"""Training-step timing (bench.py leg_train) — run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
import bench  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402

print(bench.leg_train(torch.device("cuda", 0), KerasModel.init(seed=0, randomize=True), reps=int(sys.argv[1]) if len(sys.argv) > 1 else 10))
