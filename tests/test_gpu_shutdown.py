"""Interpreter shutdown with live libavse handles: the DeviceWeights / Trainer / Context destructors hold their own
reference to the CDLL, so nothing they call at exit depends on module globals that the interpreter may already
have torn down (round 3: `AttributeError: 'NoneType' object has no attribute '_lib'` from Trainer.__del__)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
sys.path.insert(0, %r)
import avse_pkg
avse_pkg.load()
import torch
from avse_amd import ops
from avse_amd.model import KerasModel
m = KerasModel.init(seed=1, randomize=True)
dw = ops.DeviceWeights(m, "float32")
tr = ops.Trainer(m, max_batch=2)
a = torch.zeros((2, 80, 20), device="cuda")
v = torch.zeros((2, 128, 128, 5), device="cuda")
ops.forward(dw, a, v)
tr.step(a, v, a)
torch.cuda.synchronize()
# module-level references only: the interpreter tears them down in its own order at exit
keep = (dw, tr)
print("ok")
"""


@pytest.mark.gpu
def test_exit_with_live_handles_is_clean(gpu):
    r = subprocess.run([sys.executable, "-c", SCRIPT % ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("ok")
    err = [ln for ln in r.stderr.splitlines() if "amdgpu.ids" not in ln and ln.strip()]
    assert not err, "stderr at exit:\n" + "\n".join(err)
