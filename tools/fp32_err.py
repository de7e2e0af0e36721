"""Per-layer error of the fp32 forward against the float64 oracle (absolute and relative RMS, and in fp32 ulps of
each layer's RMS) on dB-scale outputs — where the north star's 1e-4 absolute RMS bound is tight.
    python tools/fp32_err.py [N] [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd import _lib, ops  # noqa: E402
from avse_amd.model import KerasModel  # noqa: E402
from oracle import keras_ref as K  # noqa: E402
from test_gpu_forward import db_scale, make_inputs, scratch  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 37
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 37
    model = db_scale(KerasModel.init(seed=seed, randomize=True))
    mel, video = make_inputs(N, seed + 100)
    inter = {}
    ref = K.forward(model.layer_dict(), mel, video, intermediates=inter)
    with _lib.context().options(unfused_tail=1):
        dw = ops.DeviceWeights(model, "float32")
        got = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
        sc = scratch(dw, N)
    eps = np.finfo(np.float32).eps
    for k in inter:
        if k not in sc:
            continue
        d = sc[k].astype(np.float64) - inter[k]
        rms = np.sqrt(np.mean(inter[k] ** 2))
        e = np.sqrt(np.mean(d ** 2))
        print(f"{k:12s} rms {rms:10.4g}  abs err {e:10.3e}  rel {e / rms:9.2e}  ({e / rms / eps:6.1f} eps)")
    e = np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2))
    print(f"{'output':12s} rms {np.sqrt(np.mean(ref ** 2)):10.4g}  abs err {e:10.3e}  rel {e / np.sqrt(np.mean(ref ** 2)):9.2e}")


if __name__ == "__main__":
    main()
