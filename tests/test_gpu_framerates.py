"""Networks for the reference's other frame rates (SURVEY.md §8(a) network build; network.py:17-40 builds from the
input shapes): at 29.97 fps preprocess_audio_signal slices [80, 24] spectrograms (n_fft 533, hop 133;
data_processor.py:44-52) with 5 video frames per slice, at 30 fps the same audio with 6 frames (:24).  Keras then
builds concat 5888 -> Dense 1472 -> ... -> dec_dense2 3840 = Reshape(5, 6, 128) (graphs pinned by
tests/golden/network_spec_2997fps.json / _30fps.json).  These shapes run the generic implicit-GEMM path for the audio
branch and the decoder (the fused per-clip audio / decoder kernels are specialised for the 25-fps grids); the video
encoder runs its own kernels at every rate (v_conv1's row-run kernel on 5 or 6 frames, the stream convolutions, whose
shapes do not change), in bf16 and in the split dtype.

Tolerances as tests/test_gpu_forward.py: fp32 relative RMS 1e-5 and absolute RMS 1e-4 on dB-scale outputs
(d_deconv6 rescaled), bf16 relative RMS 1.5e-2; training gradients as tests/test_gpu_train.py (1e-2)."""
import numpy as np
import pytest
import torch

from conftest import synth_audio, synth_video
from oracle import keras_ref as K
from oracle import keras_train_ref as KT
from oracle import librosa_ref as R
from test_gpu_forward import abs_rms, db_scale, rel_rms

pytestmark = pytest.mark.gpu

SHAPES = [(24, 5), (24, 6)]   # 29.97 fps, 30 fps


def inputs(rng, N, T, F):
    fps = 29.97 if F == 5 else 30.0
    n_fft = int(16000 / fps)
    x = synth_audio(rng, N, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, n_fft, n_fft // 4)[0][:, :T] for i in range(N)])
    return mel.astype(np.float32), synth_video(rng, N, f=F)


@pytest.mark.parametrize("T,F", SHAPES)
@pytest.mark.parametrize("dtype,N", [("float32", 3), ("float32", 37), ("float32_split", 3), ("float32_split", 37),
                                     ("bfloat16", 5)])
def test_forward_matches_oracle(gpu, T, F, dtype, N):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=T + F, randomize=True, audio_shape=(80, T), video_shape=(128, 128, F)))
    mel, video = inputs(np.random.default_rng(N), N, T, F)
    mean, std = R.video_normalizer_fit(video)
    ref = K.forward(model.layer_dict(), mel, R.video_normalize(video, mean, std).astype(np.float32))
    dw = ops.DeviceWeights(model, dtype)
    got = ops.forward(dw, ops.to_device(mel), ops.to_device(video), ops.to_device(mean), ops.to_device(std))
    got = got.cpu().numpy()
    assert got.shape == (N, 80, T)
    err, ae = rel_rms(got, ref), abs_rms(got, ref)
    print(f"T={T} F={F} {dtype} N={N}: rel {err:.2e} abs {ae:.2e} (output RMS {np.sqrt(np.mean(ref ** 2)):.3g})")
    if dtype in ("float32", "float32_split"):   # split: the fp32 bounds (tests/test_gpu_split.py)
        assert err <= 1e-5 and ae <= 1e-4, (err, ae)
    else:
        assert err <= 1.5e-2, err


@pytest.mark.parametrize("T,F", SHAPES)
def test_zero_video_and_network_api(gpu, T, F):
    """video=None (all-zero video, BASELINE configs[2]'s audio branch) and predict's squeeze at these shapes."""
    from avse_amd.network import SpeechEnhancementNetwork
    net = SpeechEnhancementNetwork.build((80, T), (128, 128, F), seed=3)
    mel, _ = inputs(np.random.default_rng(1), 4, T, F)
    ref = K.forward(net.model.layer_dict(), mel, None)
    got = net.predict_device(mel, None).cpu().numpy()
    assert rel_rms(got, ref) <= 1e-5
    one = net.predict(mel[:1], np.zeros((1, 128, 128, F), np.float32))
    assert one.shape == (80, T)


@pytest.mark.parametrize("T,F", SHAPES)
def test_training_gradients_match_oracle(gpu, T, F):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from test_gpu_train import check_gradients
    model = KerasModel.init(seed=11, randomize=True, audio_shape=(80, T), video_shape=(128, 128, F))
    rng = np.random.default_rng(2)
    mel = rng.normal(-40, 12, (3, 80, T)).astype(np.float32)
    video = rng.normal(0, 1, (3, 128, 128, F)).astype(np.float32)
    target = (mel + rng.normal(0, 3, mel.shape)).astype(np.float32)
    tr = ops.Trainer(model, max_batch=4, device=gpu)
    loss = float(tr.step(*[torch.from_numpy(a).to(gpu) for a in (mel, video, target)], dropout=0.25, seed=77,
                         grads_only=True).item())
    ref_loss, ref_g, _ = KT.gradients(model.tensors, mel, video, target, rate=0.25, seed=77)
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    check_gradients(tr.gradients(), ref_g)


@pytest.mark.parametrize("fps,F", [(29.97, 5), (30.0, 6)])
def test_enhancer_split_at_other_rates(gpu, fps, F):
    """The predict path in the default dtype at 29.97 / 30 fps: k_spec533 -> the [80, 24] network in AVSE_F32_SPLIT
    (v_conv1's row-run kernel on 5 / 6 frames, the stream convolutions) -> k_istft532, against the oracle pipeline
    per utterance (speech_enhancer.py:61-88): waveform relative RMS 1e-4 (the fp32 bound of test_enhancer_at_2997_fps)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from avse_amd.pipeline import Enhancer
    U, S = 3, 12
    rng = np.random.default_rng(int(fps * 100))
    x = synth_audio(rng, U, 3200 * S)
    video = synth_video(rng, U * S, f=F).reshape(U, S, 128, 128, F)
    mean, std = R.video_normalizer_fit(video.reshape(U * S, 128, 128, F))
    model = KerasModel.init(seed=F, randomize=True, audio_shape=(80, 24), video_shape=(128, 128, F))
    enh = Enhancer(ops.DeviceWeights(model, "float32_split"), video_frame_rate=fps, chunk=16)
    got = enh(ops.to_device(x), ops.to_device(video), ops.to_device(mean), ops.to_device(std)).cpu().numpy()
    assert enh.range_bits == 0
    for u in range(U):
        xu = R.fit_length(x[u], 3200 * S)
        sl = R.preprocess_audio_signal(xu, 16000, 200, S, fps)
        pred = K.forward(model.layer_dict(), sl.astype(np.float32),
                         R.video_normalize(video[u], mean, std).astype(np.float32))
        ref = R.reconstruct_speech_signal(xu, 16000, pred.astype(np.float32), fps)
        err = rel_rms(got[u], ref)
        print(f"{fps} fps split utterance {u}: waveform rel RMS {err:.2e}")
        assert got.shape[1] == len(ref) and err <= 1e-4, (u, err)


def test_enhancer_at_2997_fps(gpu):
    """The end-to-end predict path (pipeline.Enhancer) at 29.97 fps: K1 at n_fft 533 -> the [80, 24] network ->
    K6, against the oracle pipeline (speech_enhancer.py:61-88 per sample), fp32: waveform relative RMS 1e-4."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from avse_amd.pipeline import Enhancer
    U, S, fps = 2, 15, 29.97
    rng = np.random.default_rng(9)
    x = synth_audio(rng, U, 48000)
    video = synth_video(rng, U * S).reshape(U, S, 128, 128, 5)
    mean, std = R.video_normalizer_fit(video.reshape(U * S, 128, 128, 5))
    model = KerasModel.init(seed=4, randomize=True, audio_shape=(80, 24))
    enh = Enhancer(ops.DeviceWeights(model, "float32"), video_frame_rate=fps, chunk=8)
    got = enh(ops.to_device(x), ops.to_device(video), ops.to_device(mean), ops.to_device(std)).cpu().numpy()
    with pytest.raises(ValueError):
        Enhancer(ops.DeviceWeights(KerasModel.init(seed=0), "float32"), video_frame_rate=fps)(
            ops.to_device(x), ops.to_device(video))
    for u in range(U):
        xu = R.fit_length(x[u], 3200 * S)
        sl = R.preprocess_audio_signal(xu, 16000, 200, S, fps)
        assert sl.shape[1:] == (80, 24)
        pred = K.forward(model.layer_dict(), sl.astype(np.float32), R.video_normalize(video[u], mean, std).astype(np.float32))
        ref = R.reconstruct_speech_signal(xu, 16000, pred.astype(np.float32), fps)
        n = min(len(ref), got.shape[1])
        err = rel_rms(got[u, :n], ref[:n])
        print(f"29.97 fps utterance {u}: waveform rel RMS {err:.2e} ({got.shape[1]} vs {len(ref)} samples)")
        assert got.shape[1] == len(ref) and err <= 1e-4, (u, err)


def test_zero_video_with_layer_by_layer_audio_branch(gpu):
    """video=None with the per-layer audio encoder (no_audenc: it runs on the side stream, concurrently with the
    N = 1 encoder that computes the constant video embedding).  Round 3 found those two racing for the arena at
    29.97 fps, where the fused audio kernel does not apply; the embedding is now computed before the audio branch
    is launched.  25 fps, fp32 and bf16 against the oracle."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=5, randomize=True)
    rng = np.random.default_rng(3)
    x = synth_audio(rng, 6, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, 640, 160)[0][:, :20] for i in range(6)]).astype(np.float32)
    ref = K.forward(model.layer_dict(), mel, None)
    for dtype, tol in (("float32", 1e-5), ("bfloat16", 1.5e-2)):
        ctx = ops.DeviceWeights(model, dtype).ctx
        with ctx.options(no_audenc=1):
            dw = ops.DeviceWeights(model, dtype)
            got = ops.forward(dw, ops.to_device(mel), None).cpu().numpy()
        assert rel_rms(got, ref) <= tol, (dtype, rel_rms(got, ref))
