"""End-to-end predict path (BASELINE configs[4]; pipeline.Enhancer): whole 3-s utterances through K1 -> forward ->
K6 against the oracle pipeline (librosa restatement preprocess -> float64 Keras-semantics forward -> librosa
restatement reconstruct_speech_signal, i.e. speech_enhancer.py:61-88 per sample).

Tolerance: fp32 and fp32-split weights — the enhanced waveform within relative RMS 1e-4 of the oracle (the ISTFT's
own bound, DESIGN.md "Parity"); bf16 — the predicted mel-dB slices within MEL_BF16 and the waveform within WAVE_BF16,
each ~2x the measured error (profiles/r04a_gputest.log: mel-dB 2.65e-3, waveform 4.3e-5 relative RMS).
"""
import numpy as np
import pytest
import torch

from conftest import synth_audio, synth_video
from oracle import keras_ref as K
from oracle import librosa_ref as R

pytestmark = pytest.mark.gpu


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


def oracle_enhance(model, x, video, mean, std):
    """speech_enhancer.predict for one sample, restated on the oracle."""
    sl = R.preprocess_audio_signal(x, 16000, 200, video.shape[0], 25.0)
    vn = R.video_normalize(video, mean, std).astype(np.float32)
    pred = K.forward(model.layer_dict(), sl.astype(np.float32), vn)
    return R.reconstruct_speech_signal(x, 16000, pred.astype(np.float32), 25.0), pred


MEL_BF16, WAVE_BF16 = 6e-3, 1e-4


@pytest.mark.parametrize("dtype,n_samples", [("float32", 48000), ("float32", 47000), ("float32_split", 48000),
                                             ("bfloat16", 48000)])
def test_enhancer_matches_oracle_pipeline(gpu, dtype, n_samples):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from avse_amd.pipeline import Enhancer
    U, S = 3, 15
    rng = np.random.default_rng(5)
    x = synth_audio(rng, U, n_samples)
    video = synth_video(rng, U * S).reshape(U, S, 128, 128, 5)
    mean, std = R.video_normalizer_fit(video.reshape(U * S, 128, 128, 5))
    model = KerasModel.init(seed=8, randomize=True)
    enh = Enhancer(ops.DeviceWeights(model, dtype), chunk=16)      # chunk < U*S: several forward launches
    timings = {}
    got = enh(ops.to_device(x), ops.to_device(video), ops.to_device(mean), ops.to_device(std), timings=timings)
    got = got.cpu().numpy()
    assert got.shape == (U, 160 * (S * 20 - 1))
    assert set(timings) == {"stft_ms", "forward_ms", "istft_ms"}
    # the predicted slices of the same launch geometry (spectrogram + chunked forward), for the mel-dB bound
    sig = torch.nn.functional.pad(ops.to_device(x), (0, max(0, 3200 * S - n_samples)))[:, :3200 * S].contiguous()
    mel = ops.spectrogram(sig, frames_per_slice=20).view(U * S, 80, 20)
    pred = torch.empty_like(mel)
    frames = ops.to_device(video).view(U * S, 128, 128, 5)
    for a in range(0, U * S, 16):
        ops.forward(enh.weights, mel[a:a + 16], frames[a:a + 16], ops.to_device(mean), ops.to_device(std),
                    out=pred[a:a + 16])
    pred = pred.view(U, S, 80, 20).cpu().numpy()
    for u in range(U):
        xu = R.fit_length(x[u], 3200 * S)
        ref, ref_pred = oracle_enhance(model, xu, video[u], mean, std)
        err, perr = rel_rms(got[u], ref), rel_rms(pred[u], ref_pred)
        print(f"{dtype} utterance {u}: waveform rel RMS {err:.3e}, predicted mel-dB rel RMS {perr:.3e}")
        if dtype == "bfloat16":
            assert perr <= MEL_BF16 and err <= WAVE_BF16, (u, perr, err)
        else:
            assert err <= 1e-4 and perr <= 1e-5, (u, err, perr)


def test_enhancer_rejects_mismatched_geometry(gpu):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from avse_amd.pipeline import Enhancer
    enh = Enhancer(ops.DeviceWeights(KerasModel.init(seed=0), "float32"))
    sig = torch.zeros((2, 48000), device="cuda")
    with pytest.raises(ValueError):
        enh(sig, torch.zeros((3, 15, 128, 128, 5), device="cuda"))


def test_enhancer_split_1024_chunks_many_utterances(gpu):
    """The credited dtype end to end at the bench's e2e geometry (bench.py --e2e: forward chunks of 1024 clips): 72
    3-s utterances (1,080 clips: one full 1024-clip chunk and a ragged 56-clip one) through K1 -> split forward ->
    K6 in one Enhancer call; utterances on both sides of the chunk boundary and at the ends against the oracle pipeline
    (speech_enhancer.py:61-88 per sample, float64 forward)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from avse_amd.pipeline import Enhancer
    U, S = 72, 15
    rng = np.random.default_rng(72)
    x = synth_audio(rng, U, 48000)
    video = synth_video(rng, U * S).reshape(U, S, 128, 128, 5)
    mean, std = R.video_normalizer_fit(video.reshape(U * S, 128, 128, 5))
    model = KerasModel.init(seed=21, randomize=True)
    dw = ops.DeviceWeights(model, "float32_split")
    enh = Enhancer(dw, chunk=1024)
    got = enh(ops.to_device(x), ops.to_device(video), ops.to_device(mean), ops.to_device(std)).cpu().numpy()
    assert got.shape == (U, 160 * (S * 20 - 1)) and np.isfinite(got).all()
    assert enh.range_bits == 0
    for u in (0, 1, 1023 // S, 1024 // S, 1025 // S, U - 1):     # utterance 68 straddles clips 1020..1034
        ref, _ = oracle_enhance(model, x[u], video[u], mean, std)
        err = rel_rms(got[u], ref)
        print(f"split e2e utterance {u}: waveform rel RMS {err:.3e}")
        assert err <= 1e-4, (u, err)
