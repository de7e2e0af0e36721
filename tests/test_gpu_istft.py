"""K6 parity: libavse ISTFT reconstruction vs the numpy librosa restatement.

Tolerance (DESIGN.md "Parity"): the reconstructed waveform within relative RMS 1e-4 of the float64
oracle (fp32 exp10 / pinv dot / inverse FFT / overlap-add); output length exact.
"""
import numpy as np
import pytest
import torch

from conftest import synth_audio
from oracle import librosa_ref as R

pytestmark = pytest.mark.gpu


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


@pytest.mark.parametrize("n_samples,fps,n_slices", [(48000, 25.0, 15), (47000, 25.0, 15), (32000, 29.97, 10)])
def test_reconstruct_speech_signal_matches_oracle(gpu, n_samples, fps, n_slices):
    from avse_amd import data_processor as dp
    from avse_amd.audio_io import AudioSignal
    rng = np.random.default_rng(7)
    x = synth_audio(rng, 1, n_samples)[0]
    sig = AudioSignal(x.copy(), 16000)
    slices = dp.preprocess_audio_signal(sig, 200, n_slices, fps)            # pads/truncates sig in place
    # a "prediction": the speech slices perturbed a little (as a network output would be)
    pred = (slices + rng.normal(0, 1.0, slices.shape)).astype(np.float32)
    got = dp.reconstruct_speech_signal(sig, pred, fps).get_data(0)
    ref = R.reconstruct_speech_signal(sig.get_data(0), 16000, pred, fps)
    assert got.shape == ref.shape
    g = R.frame_geometry(16000, 200, n_slices, fps)
    assert got.shape[0] == g["hop_length"] * (n_slices * g["spectrogram_samples_per_slice"] - 1)
    assert rel_rms(got, ref) < 1e-4, rel_rms(got, ref)


def test_batched_istft_matches_oracle(gpu):
    from avse_amd import ops
    rng = np.random.default_rng(3)
    x = synth_audio(rng, 5, 48000)
    xt = torch.from_numpy(x).to(gpu)
    mel, D = ops.spectrogram(xt, frames_per_slice=20, return_stft=True)     # [5, 15, 80, 20], [5, 321, 301]
    y = ops.istft(mel, D).cpu().numpy()
    assert y.shape == (5, 47840)
    for u in range(5):
        sl = R.preprocess_audio_signal(x[u], 16000, 200, 15, 25.0)
        ref = R.reconstruct_speech_signal(x[u], 16000, sl, 25.0)
        assert rel_rms(y[u], ref) < 1e-4, (u, rel_rms(y[u], ref))


def test_fused_istft_at_e2e_size_matches_oracle(gpu):
    """The ISTFT launch of BASELINE configs[4] (bench.py --e2e): 667 3-s utterances (10,005 clips) in ONE avse_istft
    call — every persistent block walks many output chunks — each utterance against the oracle's
    reconstruct_speech_signal.  The input is a perturbed copy of the mixture's own slices (a network-like
    prediction), so amplitudes span the whole dB range."""
    from avse_amd import ops
    U = 667
    rng = np.random.default_rng(667)
    x = synth_audio(rng, U, 48000)
    xt = torch.from_numpy(x).to(gpu)
    mel, D = ops.spectrogram(xt, frames_per_slice=20, return_stft=True)     # [667, 15, 80, 20], [667, 321, 301]
    pred = mel + torch.from_numpy(rng.normal(0, 1.0, tuple(mel.shape)).astype(np.float32)).to(gpu)
    y = ops.istft(pred, D).cpu().numpy()
    assert y.shape == (U, 47840)
    assert np.isfinite(y).all()
    pred_np = pred.cpu().numpy()
    worst = 0.0
    for u in range(U):
        ref = R.reconstruct_speech_signal(x[u], 16000, pred_np[u], 25.0)
        worst = max(worst, rel_rms(y[u], ref))
    print(f"ISTFT 667 utterances: worst waveform rel RMS {worst:.3e}")
    assert worst < 1e-4, worst


def test_reconstruct_signal_from_spectrogram_api(gpu):
    from avse_amd import data_processor as dp
    from avse_amd.audio_io import AudioSignal
    rng = np.random.default_rng(4)
    x = synth_audio(rng, 1, 16000)[0]
    mel, phase = dp.signal_to_spectrogram(AudioSignal(x, 16000), 640, 160)
    got = dp.reconstruct_signal_from_spectrogram(mel, phase, 16000, 640, 160).get_data(0)
    mref, pref = R.signal_to_spectrogram(x, 16000, 640, 160)
    ref = R.reconstruct_signal_from_spectrogram(mref, pref, 16000, 640, 160)
    assert got.shape == ref.shape == (16000,)
    assert rel_rms(got, ref) < 1e-4, rel_rms(got, ref)


@pytest.mark.parametrize("n_samples", [48000, 47000, 3200])
def test_fused_istft_matches_dense_path(gpu, n_samples):
    """k_istft_fused (tridiagonal Gram solve + in-LDS overlap-add) against the dense-pinv / scratch-frame /
    k_ola path on the same inputs, including a chunk that ends mid-block (47000) and a one-chunk signal."""
    from avse_amd import _lib, ops
    rng = np.random.default_rng(11)
    x = torch.from_numpy(synth_audio(rng, 3, n_samples)).to(gpu)
    mel, D = ops.spectrogram(x, frames_per_slice=20, return_stft=True)
    pred = mel + torch.from_numpy(rng.normal(0, 1.0, tuple(mel.shape)).astype(np.float32)).to(gpu)
    fused = ops.istft(pred, D)
    with _lib.context(gpu).options(dense_istft=1):
        dense = ops.istft(pred, D)
    torch.cuda.synchronize()
    assert fused.shape == dense.shape
    assert rel_rms(fused.cpu().numpy(), dense.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("U,n_samples", [(24, 48000), (3, 3200)])
def test_batched_istft_533_matches_oracle(gpu, U, n_samples):
    """29.97 / 30 fps (analysis n_fft 533, hop 133: the inverse is 532 = 28 x 19, k_istft532) on a batch of 3-s
    utterances (361 frames, 23 chunks of 16) and on 200-ms segments (25 frames, a partial chunk), perturbed
    predictions, each utterance against the oracle's reconstruct_speech_signal."""
    from avse_amd import ops
    rng = np.random.default_rng(533 + U)
    x = synth_audio(rng, U, n_samples)
    xt = torch.from_numpy(x).to(gpu)
    mel, D = ops.spectrogram(xt, n_fft=533, hop_length=133, frames_per_slice=24, return_stft=True)
    pred = mel + torch.from_numpy(rng.normal(0, 1.0, tuple(mel.shape)).astype(np.float32)).to(gpu)
    y = ops.istft(pred, D, n_fft=533, hop_length=133).cpu().numpy()
    ns = n_samples // 3200
    assert y.shape == (U, 133 * (24 * ns - 1))
    pred_np = pred.cpu().numpy()
    worst = 0.0
    for u in range(U):
        ref = R.reconstruct_speech_signal(x[u], 16000, pred_np[u], 29.97)
        assert ref.shape == y[u].shape
        worst = max(worst, rel_rms(y[u], ref))
    print(f"ISTFT n_fft 533, {U} x {n_samples} samples: worst waveform rel RMS {worst:.3e}")
    assert worst < 1e-4, worst
