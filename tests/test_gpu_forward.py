"""K2-K5 parity: libavse forward vs the Keras-semantics oracle (oracle/keras_ref.py, float64).

Tolerances (DESIGN.md "Parity"):
  fp32 path  — relative RMS  ||gpu - ref||_2 / ||ref||_2 <= 1e-5 and absolute RMS <= 1e-4 x max(1, RMS(ref))
               (the north star's "enhanced magnitude within 1e-4 RMS"; exact-fp32 MFMA, fp32 accumulation)
  bf16 path  — relative RMS <= 3e-2 (bf16 operands, fp32 accumulation; SURVEY.md §7 "Tolerance vs bf16")
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import synth_video
from oracle import keras_ref as K
from oracle import librosa_ref as R

pytestmark = pytest.mark.gpu

BUF_NAMES = ["video_in", "audio_in", "a_conv1", "a_conv2", "a_conv3", "a_conv4", "v_conv1", "v_conv2", "v_conv3",
             "v_conv4", "v_conv5", "concat", "enc_dense", "dec_dense1", "dec_dense2", "d_deconv1", "d_deconv2",
             "d_deconv3", "d_deconv4", "d_deconv5"]
BUF_SHAPES = {"video_in": (128, 128, 8), "audio_in": (80, 20, 8), "a_conv1": (40, 10, 64), "a_conv2": (40, 10, 64),
              "a_conv3": (20, 5, 128), "a_conv4": (10, 5, 128), "v_conv1": (64, 64, 128), "v_conv2": (32, 32, 128),
              "v_conv3": (16, 16, 256), "v_conv4": (8, 8, 256), "v_conv5": (4, 4, 512), "concat": (5248,),
              "enc_dense": (1312,), "dec_dense1": (1312,), "dec_dense2": (5, 5, 128), "d_deconv1": (10, 5, 128),
              "d_deconv2": (20, 5, 128), "d_deconv3": (40, 10, 128), "d_deconv4": (40, 10, 64),
              "d_deconv5": (80, 20, 64)}


def make_inputs(N, seed):
    rng = np.random.default_rng(seed)
    from conftest import synth_audio
    x = synth_audio(rng, N, 3200)
    mel = np.stack([R.signal_to_spectrogram(x[i], 16000, 640, 160)[0][:, :20] for i in range(N)]).astype(np.float32)
    video = synth_video(rng, N)
    return mel, video


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def scratch(dw, N):
    """Read libavse's intermediate activations (avse_debug_scratch) as float32 numpy arrays."""
    from avse_amd import _lib
    base = ctypes.c_void_p()
    offs = (ctypes.c_int64 * 20)()
    _lib.check(_lib.load().avse_debug_scratch(dw.ctx.handle, N, dw.dtype, ctypes.byref(base), offs), "debug")
    dt = torch.bfloat16 if dw.dtype == _lib.AVSE_BF16 else torch.float32
    es = 2 if dw.dtype == _lib.AVSE_BF16 else 4
    out = {}
    torch.cuda.synchronize()
    for i, name in enumerate(BUF_NAMES):
        n = N * int(np.prod(BUF_SHAPES[name]))
        t = torch.empty(n, dtype=dt, device="cuda")
        from avse_amd import _lib as L
        hip = ctypes.CDLL("libamdhip64.so.7")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        rc = hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(base.value + offs[i]), n * es, 3)
        assert rc == 0
        out[name] = t.float().cpu().numpy().reshape((N,) + BUF_SHAPES[name])
    return out


def run_case(gpu, N, dtype, seed=0, normalize=False):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=seed, randomize=True)
    mel, video = make_inputs(N, seed + 100)
    mean = std = None
    vref = video
    if normalize:
        mean, std = R.video_normalizer_fit(video)
        vref = R.video_normalize(video, mean, std).astype(np.float32)
    inter = {}
    ref = K.forward(model.layer_dict(), mel, vref, intermediates=inter)
    dw = ops.DeviceWeights(model, dtype)
    args = [ops.to_device(mel), ops.to_device(video)]
    if normalize:
        args += [ops.to_device(mean), ops.to_device(std)]
    got = ops.forward(dw, *args).cpu().numpy()
    return got, ref, inter, dw


@pytest.mark.parametrize("N", [1, 3, 37])
def test_forward_fp32_matches_oracle(gpu, N):
    got, ref, inter, dw = run_case(gpu, N, "float32", seed=N)
    err = rel_rms(got, ref)
    abs_rms = float(np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2)))
    if err > 1e-5:
        sc = scratch(dw, N)
        report = {k: rel_rms(sc[k], inter[k]) for k in inter if k in sc}
        pytest.fail(f"rel RMS {err:.3e}; per-layer rel RMS: {report}")
    assert abs_rms <= 1e-4 * max(1.0, float(np.sqrt(np.mean(ref ** 2)))), abs_rms


def test_forward_fp32_fused_normalizer(gpu):
    got, ref, inter, dw = run_case(gpu, 4, "float32", seed=7, normalize=True)
    assert rel_rms(got, ref) <= 1e-5


@pytest.mark.parametrize("N", [2, 130])
def test_forward_bf16_matches_oracle(gpu, N):
    got, ref, inter, dw = run_case(gpu, N, "bfloat16", seed=11 + N, normalize=True)
    err = rel_rms(got, ref)
    if err > 3e-2:
        sc = scratch(dw, N)
        report = {k: rel_rms(sc[k], inter[k]) for k in inter if k in sc}
        pytest.fail(f"rel RMS {err:.3e}; per-layer rel RMS: {report}")


@pytest.mark.parametrize("N", [1, 5])
def test_bf16_halo_video_convs_match_generic_kernel(gpu, N, monkeypatch):
    """The halo-tiled video convs (conv_halo.hip) against the generic implicit-GEMM kernel and the
    oracle, layer by layer (N=5 exercises the 4-clip tiles of v_conv5 with a ragged last tile)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=3, randomize=True)
    mel, video = make_inputs(N, 9)
    mean, std = R.video_normalizer_fit(video)
    args = [ops.to_device(mel), ops.to_device(video), ops.to_device(mean), ops.to_device(std)]
    inter = {}
    ref = K.forward(model.layer_dict(), mel, R.video_normalize(video, mean, std).astype(np.float32), intermediates=inter)
    dw_h = ops.DeviceWeights(model, "bfloat16")
    out_h = ops.forward(dw_h, *args).cpu().numpy()
    sc_h = scratch(dw_h, N)
    monkeypatch.setenv("AVSE_NO_HALO", "1")
    dw_g = ops.DeviceWeights(model, "bfloat16")
    out_g = ops.forward(dw_g, *args).cpu().numpy()
    sc_g = scratch(dw_g, N)
    for k in ["v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5"]:
        assert rel_rms(sc_h[k], inter[k]) <= 1.5e-2, (k, rel_rms(sc_h[k], inter[k]))
        assert rel_rms(sc_h[k], sc_g[k]) <= 1.5e-2, (k, rel_rms(sc_h[k], sc_g[k]))
    assert rel_rms(out_h, ref) <= 3e-2
    assert rel_rms(out_h, out_g) <= 3e-2


def test_intermediates_fp32(gpu, monkeypatch):
    """Every layer's activation, not only the output, matches the oracle (catches compensating bugs).
    d_deconv6 runs unfused here so the d_deconv5 activation is materialised; the fused path is covered by
    every output comparison and by test_fused_tail_matches_unfused."""
    monkeypatch.setenv("AVSE_UNFUSED_TAIL", "1")
    got, ref, inter, dw = run_case(gpu, 2, "float32", seed=21)
    sc = scratch(dw, 2)
    for k in inter:
        if k in sc:
            assert rel_rms(sc[k], inter[k]) <= 1e-5, (k, rel_rms(sc[k], inter[k]))


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-6), ("bfloat16", 2e-3)])
def test_fused_tail_matches_unfused(gpu, monkeypatch, dtype, tol):
    """d_deconv5 + d_deconv6 fused (the 64 -> 1 dot in d_deconv5's epilogue) against the two-kernel path;
    both round the d_deconv5 activation to the compute dtype, only the summation order differs."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=4, randomize=True)
    mel, video = make_inputs(7, 44)
    args = [ops.to_device(mel), ops.to_device(video)]
    dw = ops.DeviceWeights(model, dtype)
    fused = ops.forward(dw, *args).cpu().numpy()
    monkeypatch.setenv("AVSE_UNFUSED_TAIL", "1")
    unfused = ops.forward(dw, *args).cpu().numpy()
    assert rel_rms(fused, unfused) <= tol, rel_rms(fused, unfused)


def test_predict_and_evaluate_single_forward(gpu):
    """The CLI's one-forward predict prints the loss evaluate() reports (speech_enhancer.py:76-79)."""
    from avse_amd.network import SpeechEnhancementNetwork
    net = SpeechEnhancementNetwork.build((80, 20), (128, 128, 5), seed=3)
    mel, video = make_inputs(4, 8)
    target = np.random.default_rng(1).normal(size=mel.shape).astype(np.float32)
    pred, loss = net.predict_and_evaluate(mel, video, target)
    assert np.array_equal(pred, net.predict(mel, video))
    assert abs(loss - net.evaluate(mel, video, target)) <= 1e-6 * abs(loss)
    assert abs(loss - K.mse(pred[:, :, :], target)) <= 1e-5 * abs(loss)


def test_mse_matches(gpu):
    from avse_amd import ops
    rng = np.random.default_rng(0)
    a = rng.normal(size=(5, 80, 20)).astype(np.float32)
    b = rng.normal(size=(5, 80, 20)).astype(np.float32)
    got = float(ops.mse(ops.to_device(a), ops.to_device(b)).item())
    assert abs(got - K.mse(a, b)) <= 1e-6 * K.mse(a, b)


def test_network_api_shapes(gpu):
    from avse_amd.network import SpeechEnhancementNetwork
    net = SpeechEnhancementNetwork.build((80, 20), (128, 128, 5))
    mel, video = make_inputs(3, 5)
    assert net.predict(mel, video).shape == (3, 80, 20)
    assert net.predict(mel[:1], video[:1]).shape == (80, 20)      # np.squeeze quirk (network.py:212)
    loss = net.evaluate(mel, video, mel)
    assert isinstance(loss, float) and np.isfinite(loss)


@pytest.mark.parametrize("env", ["AVSE_V1_IM2COL", "AVSE_MFMA32"])
def test_bf16_video_kernel_variants_agree(gpu, env, monkeypatch):
    """A/B kernel variants of the bf16 video encoder (conv_v1r.hip kernel-row runs vs conv_v1.hip dense
    im2col; 16x16x32 vs 32x32x16 stream-conv compute waves) give the same layer outputs and match the oracle."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    N = 3
    model = KerasModel.init(seed=5, randomize=True)
    mel, video = make_inputs(N, 21)
    mean, std = R.video_normalizer_fit(video)
    args = [ops.to_device(mel), ops.to_device(video), ops.to_device(mean), ops.to_device(std)]
    inter = {}
    K.forward(model.layer_dict(), mel, R.video_normalize(video, mean, std).astype(np.float32), intermediates=inter)
    dw = ops.DeviceWeights(model, "bfloat16")
    out_a = ops.forward(dw, *args).cpu().numpy()
    sc_a = scratch(dw, N)
    monkeypatch.setenv(env, "1")
    out_b = ops.forward(dw, *args).cpu().numpy()
    sc_b = scratch(dw, N)
    for k in ["v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5"]:
        assert rel_rms(sc_a[k], inter[k]) <= 1.5e-2, (k, rel_rms(sc_a[k], inter[k]))
        assert rel_rms(sc_a[k], sc_b[k]) <= 1e-2, (k, rel_rms(sc_a[k], sc_b[k]))
    assert rel_rms(out_a, out_b) <= 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 5, 37])
def test_bf16_fused_per_clip_kernels_match_layer_path(gpu, N, monkeypatch):
    """The per-clip fused kernels (conv_aud.hip: a_conv1..a_conv5; conv_dech.hip: d_deconv1..d_deconv3; conv_dec.hip:
    d_deconv4..d_deconv6) and gemm.hip (v_conv6, dense) against the layer-by-layer k_conv launches
    (AVSE_NO_AUDENC / AVSE_NO_DECHEAD / AVSE_NO_DECTAIL / AVSE_NO_GEMM = 1) and the float64 oracle: the audio
    embedding (concat[0:3200]) and the network output.  Both paths round every activation to bf16, so they differ
    only in fp32 summation order."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=11, randomize=True)
    mel, video = make_inputs(N, 31)
    mean, std = R.video_normalizer_fit(video)
    args = [ops.to_device(mel), ops.to_device(video), ops.to_device(mean), ops.to_device(std)]
    inter = {}
    ref = K.forward(model.layer_dict(), mel, R.video_normalize(video, mean, std).astype(np.float32), intermediates=inter)
    dw = ops.DeviceWeights(model, "bfloat16")
    out_f = ops.forward(dw, *args).cpu().numpy()
    cat_f = scratch(dw, N)["concat"][:, :3200].copy()
    for env in ("AVSE_NO_AUDENC", "AVSE_NO_DECHEAD", "AVSE_NO_DECTAIL", "AVSE_NO_GEMM"):
        monkeypatch.setenv(env, "1")
    out_l = ops.forward(dw, *args).cpu().numpy()
    cat_l = scratch(dw, N)["concat"][:, :3200].copy()
    assert rel_rms(cat_f, cat_l) <= 1e-2, rel_rms(cat_f, cat_l)
    assert rel_rms(out_f, out_l) <= 1e-2, rel_rms(out_f, out_l)
    assert rel_rms(out_f.reshape(ref.shape), ref) <= 3e-2, rel_rms(out_f.reshape(ref.shape), ref)


@pytest.mark.gpu
def test_forward_graph_replay(gpu, monkeypatch):
    """avse_forward's hipGraph cache: the first call with an argument set launches directly, the second captures, later
    ones replay — with new input CONTENTS at the same addresses the replay computes on them (bit-identical to direct
    launches), and a changed AVSE_* switch or N gets its own entry (AVSE_GRAPH=1 enables the cache)."""
    import torch
    from avse_amd import ops
    from avse_amd.model import KerasModel
    N = 7
    model = KerasModel.init(seed=5, randomize=True)
    dw = ops.DeviceWeights(model, "bfloat16")
    mel0, video0 = make_inputs(N, 3)
    mean, std = R.video_normalizer_fit(video0)
    d = [ops.to_device(mel0), ops.to_device(video0), ops.to_device(mean), ops.to_device(std)]
    out = torch.empty((N, 80, 20), dtype=torch.float32, device=d[0].device)
    monkeypatch.setenv("AVSE_GRAPH", "1")
    results = []
    for seed in (3, 4, 5, 6):   # direct, capture, replay, replay
        mel, video = make_inputs(N, seed)
        d[0].copy_(torch.from_numpy(mel.reshape(d[0].shape)))
        d[1].copy_(torch.from_numpy(video.reshape(d[1].shape)))
        ops.forward(dw, *d, out=out)
        results.append(out.cpu().numpy().copy())
    monkeypatch.delenv("AVSE_GRAPH")
    for k, seed in enumerate((3, 4, 5, 6)):
        mel, video = make_inputs(N, seed)
        d[0].copy_(torch.from_numpy(mel.reshape(d[0].shape)))
        d[1].copy_(torch.from_numpy(video.reshape(d[1].shape)))
        ops.forward(dw, *d, out=out)
        np.testing.assert_array_equal(out.cpu().numpy(), results[k])
    assert not np.array_equal(results[2], results[3])
