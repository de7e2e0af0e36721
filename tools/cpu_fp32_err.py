"""Error of a CPU float32 framework forward (torch-CPU float32 running the oracle's Keras-semantics graph, the stand-in
for the reference's Keras/TF-CPU float32 model) against the float64 oracle, on the GPU suite's hardest parity case
(tests/test_gpu_split.py: N clips, seed N, dB-scale output layer):   python tools/cpu_fp32_err.py [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd.model import KerasModel  # noqa: E402
from oracle import keras_ref as K  # noqa: E402
from test_gpu_forward import db_scale, make_inputs  # noqa: E402

if __name__ == "__main__":
    torch.set_num_threads(8)
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 37
    m = db_scale(KerasModel.init(seed=N, randomize=True))
    mel, video = make_inputs(N, N + 100)
    wd = m.layer_dict()
    ref = K.forward(wd, mel, video)
    got = K.forward(wd, mel, video, dtype=torch.float32)
    print(f"N={N}: torch-CPU float32 abs RMS error {np.sqrt(np.mean((got - ref) ** 2)):.3e} "
          f"(output RMS {np.sqrt(np.mean(ref ** 2)):.3g})")
