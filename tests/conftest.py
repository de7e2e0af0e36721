import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import avse_pkg  # noqa: E402

avse_pkg.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and libavse.so")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    # Only -m gpu tests request this fixture.  A GPU run on a box where torch sees no device must FAIL, not skip:
    # an all-skipped `pytest -m gpu` would exit 0 without having run a single kernel.
    if not has_gpu():
        pytest.fail("no ROCm GPU visible to torch: the -m gpu tests cannot run here", pytrace=False)
    import torch
    return torch.device("cuda", 0)


def synth_audio(rng, n_utt, n_samples, sr=16000):
    """int16-scale gaussian noise + a 200-3000 Hz harmonic component."""
    t = np.arange(n_samples) / sr
    out = np.empty((n_utt, n_samples), dtype=np.float32)
    for u in range(n_utt):
        f0 = rng.uniform(200, 3000)
        harm = sum((3000.0 / (h + 1)) * np.sin(2 * np.pi * f0 * (h + 1) * t + rng.uniform(0, 2 * np.pi))
                   for h in range(3))
        noise = rng.normal(0, 3000, n_samples)
        out[u] = np.clip(np.round(noise + harm), -32768, 32767)
    return out


def synth_video(rng, n, h=128, w=128, f=5):
    return rng.integers(0, 256, size=(n, h, w, f)).astype(np.float32)
