"""Checked build on the GPU (SURVEY §5 race detection / sanitizers): tests/native/abi_checked links the library
compiled with -DAVSE_DEBUG (device-side protocol and bounds checks: v_conv1's window-slot tags at both ends of every
tile, the segment STFT's LDS-DMA staging against the utterance's samples, k_spec640's output bounds, the fused ISTFT's
chunk frame window and overlap-add reads) and with AddressSanitizer on the host code, and drives the C-ABI through
the STFT (both kernels), the ISTFT, the bf16 forward at N = 300 (75 v_conv1 tiles per persistent workgroup: the
three-slot window ring wraps 25 times), the fp32 forward, the all-zero-video path and one training step.  Any check
that fires makes the call return AVSE_ERR_CHECK with the record in avse_last_error; the harness exits non-zero."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_checked_build_harness_on_device(gpu):
    exe = os.path.join(ROOT, "tests", "native", "abi_checked")
    assert os.path.exists(exe), "tests/native/abi_checked is not built (make -C .../csrc checked)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "gpu part run" in r.stdout and "ok: 0 failure(s)" in r.stdout, r.stdout
