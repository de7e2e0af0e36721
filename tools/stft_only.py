"""configs[1] STFT leg alone (bench.leg_stft), for rocprofv3 passes: python tools/stft_only.py [reps] [lib]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import avse_pkg  # noqa: E402

avse_pkg.load()
if len(sys.argv) > 2:
    sys.modules["avse_amd"]._lib.LIB_PATH = os.path.abspath(sys.argv[2])
import torch  # noqa: E402

import bench  # noqa: E402

print(bench.leg_stft(torch.device("cuda", 0), reps=int(sys.argv[1]) if len(sys.argv) > 1 else 20))
