"""K1 / K6 while matrix-core work of another kernel shares the CUs (round 5).

On gfx950 `v_pk_add_f32` with a half-swapping op_sel on its second source returned wrong values in lanes 48..63 when
MFMA work of another kernel ran beside it (tools/pk_probe.py); the round-4 STFT helpers used that form, so a spectrogram
launched on one stream while an MFMA loop (or the split forward) ran on another came back with one frame per wave
wrong in most runs (36 of 36 beside an MFMA loop; 14 of 36 beside the split forward).  The helpers are now one
v_pk_fma_f32 each.  These tests run each transform alone for a reference, then beside tests/native/libcobusy.so's MFMA
loop on a second stream, and require bit-identical outputs (the transforms are deterministic)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import synth_audio

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPS, ITERS = 6, 20


def _cobusy():
    path = os.path.join(ROOT, "tests", "native", "libcobusy.so")
    if not os.path.exists(path):
        pytest.fail("tests/native/libcobusy.so is missing: build it with `make -C audio-visual-speech-enhancement_amd/csrc "
                    "cobusy` (__graft_entry__.build does)")
    return ctypes.CDLL(path)


def _beside_mfma(gpu, fn):
    """fn() alone, then REPS x ITERS times beside the MFMA loop on a second stream: the number of reps whose last
    output differs from the solo one."""
    lib = _cobusy()
    busy = torch.empty(4096 * 256, dtype=torch.float32, device=gpu)
    side = torch.cuda.Stream(gpu)
    ref = fn().clone()
    torch.cuda.synchronize()
    bad = 0
    for _ in range(REPS):
        for _ in range(ITERS):
            assert lib.cobusy_launch(ctypes.c_void_p(busy.data_ptr()), 4096, 2000, ctypes.c_void_p(side.cuda_stream)) == 0
            out = fn()
        torch.cuda.synchronize()
        bad += int(not torch.equal(out, ref))
    return bad


@pytest.mark.parametrize("n_fft,hop,spf,L,stft", [(640, 160, 20, 3200, False), (533, 133, 24, 3200, False),
                                                 (640, 160, 20, 48000, True), (533, 133, 24, 48000, True)])
def test_spectrogram_beside_matrix_core_work(gpu, n_fft, hop, spf, L, stft):
    """200-ms segments (k_spec_seg / k_spec533 in one block) and 3-s utterances with the complex STFT (k_spec640 /
    k_spec533 chunked + the top_db clamp pass)."""
    from avse_amd import ops
    x = torch.from_numpy(synth_audio(np.random.default_rng(21), 512 if L == 3200 else 32, L)).to(gpu)

    def run():
        r = ops.spectrogram(x, n_fft=n_fft, hop_length=hop, frames_per_slice=spf, return_stft=stft)
        return torch.cat([r[0].flatten(), torch.view_as_real(r[1]).flatten()]) if stft else r

    bad = _beside_mfma(gpu, run)
    print(f"n_fft {n_fft}, {L} samples: {bad} of {REPS} reps differ from the solo spectrogram")
    assert bad == 0


@pytest.mark.parametrize("n_fft,hop,spf", [(640, 160, 20), (533, 133, 24)])
def test_istft_beside_matrix_core_work(gpu, n_fft, hop, spf):
    from avse_amd import ops
    x = torch.from_numpy(synth_audio(np.random.default_rng(22), 32, 48000)).to(gpu)
    mel, D = ops.spectrogram(x, n_fft=n_fft, hop_length=hop, frames_per_slice=spf, return_stft=True)
    bad = _beside_mfma(gpu, lambda: ops.istft(mel, D, n_fft=n_fft, hop_length=hop))
    print(f"n_fft {n_fft}: {bad} of {REPS} reps differ from the solo ISTFT")
    assert bad == 0
