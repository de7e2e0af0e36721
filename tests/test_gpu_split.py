"""AVSE_F32_SPLIT parity: the video convolutions on split-f16 operands (conv_v1r.hip k_conv_v1s, conv_stream.hip
k_conv_stream<..., S16>: every fp32 operand as the f16 pair h + l, all four products on the 16-bit matrix cores,
fp32 accumulation) against the float64 Keras-semantics oracle, under the SAME bounds as the exact-fp32 path
(test_gpu_forward.py FP32_ABS / FP32_REL: the north star's 1e-4 absolute RMS on dB-scale outputs, 1e-5 relative),
every materialised layer included; and against the exact-fp32 path's own error (measured: no worse).
"""
import numpy as np
import pytest

from oracle import keras_ref as K
from oracle import librosa_ref as R
from test_gpu_forward import (FP32_ABS, FP32_REL, abs_rms, db_scale, make_inputs, rel_rms, run_case, scratch,
                              spread_clips)

pytestmark = pytest.mark.gpu

SPLIT = "float32_split"


@pytest.mark.parametrize("N,db", [(1, False), (3, True), (37, False), (37, True)])
def test_split_forward_matches_oracle(gpu, N, db):
    got, ref, inter, dw = run_case(gpu, N, SPLIT, seed=N, db=db)
    err, ae = rel_rms(got, ref), abs_rms(got, ref)
    got32, _, _, _ = run_case(gpu, N, "float32", seed=N, db=db)
    ae32 = abs_rms(got32, ref)
    print(f"split N={N} db={db}: output RMS {np.sqrt(np.mean(ref ** 2)):.3g}, abs RMS err {ae:.3e} (exact fp32 "
          f"{ae32:.3e}), rel {err:.3e}")
    if err > FP32_REL:
        sc = scratch(dw, N)
        report = {k: rel_rms(sc[k], inter[k]) for k in inter if k in sc}
        pytest.fail(f"rel RMS {err:.3e}; per-layer rel RMS: {report}")
    assert ae <= FP32_ABS, ae
    assert ae <= 1.5 * ae32 + 1e-6, (ae, ae32)


def test_split_intermediates(gpu):
    """Every layer (the split-pair buffers decoded h + l) against the oracle; the fused d_deconv6 is unfused here."""
    from avse_amd import _lib
    with _lib.context().options(unfused_tail=1):   # every decoder layer materialised
        got, ref, inter, dw = run_case(gpu, 2, SPLIT, seed=21, normalize=True)
        sc = scratch(dw, 2)
    for k in inter:
        if k in sc:
            print(f"{k:12s} rel {rel_rms(sc[k], inter[k]):.2e}")
            assert rel_rms(sc[k], inter[k]) <= FP32_REL, (k, rel_rms(sc[k], inter[k]))


@pytest.mark.parametrize("N", [5, 301, 512, 1024])
def test_split_bench_batch_matches_oracle(gpu, N):
    """The launch bench.py times in the split dtype (its inputs, normaliser, 512 clips; N = 301 and 5 leave ragged
    4-clip v_conv5 tiles; N = 1024 is the forward chunk of the end-to-end configs[4] run, pipeline.Enhancer): output and
    every materialised layer of spread clips against the float64 oracle."""
    import bench
    from avse_amd import ops
    from avse_amd.model import KerasModel
    rng = np.random.default_rng(1234)
    audio_np, video_np = bench.synth(rng, N)
    mean_np = video_np.mean(axis=(0, 3)).astype(np.float32)
    std_np = video_np.std(axis=(0, 3)).astype(np.float32)
    model = db_scale(KerasModel.init(seed=0, randomize=True))
    dw = ops.DeviceWeights(model, SPLIT)
    mel = ops.spectrogram(ops.to_device(audio_np), frames_per_slice=20).view(N, 80, 20)
    out = ops.forward(dw, mel, ops.to_device(video_np), ops.to_device(mean_np), ops.to_device(std_np)).cpu().numpy()
    clips = spread_clips(N, k=12)
    mel_np = mel.cpu().numpy()[clips]
    inter = {}
    vn = R.video_normalize(video_np[clips], mean_np, std_np).astype(np.float32)
    ref = K.forward(model.layer_dict(), mel_np, vn, intermediates=inter)
    # d_deconv4's output lives only in LDS in the fused split tail (conv_dects.hip): it is checked layer by layer in
    # test_split_intermediates and against the layer path in test_split_fused_tail_matches_layer_path
    names = ["v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5", "concat", "enc_dense", "dec_dense1", "dec_dense2",
             "d_deconv1", "d_deconv2", "d_deconv3"]
    sc = scratch(dw, N, clips, names)
    layers = {k: rel_rms(sc[k], inter[k]) for k in names}
    ae = abs_rms(out[clips], ref)
    print(f"split N={N}: output abs RMS {ae:.3e} rel {rel_rms(out[clips], ref):.3e}; per layer {layers}")
    assert np.isfinite(out).all()
    assert ae <= FP32_ABS
    assert rel_rms(out[clips], ref) <= FP32_REL
    for k, e in layers.items():
        assert e <= FP32_REL, (k, e)


@pytest.mark.parametrize("N", [120, 256])
def test_split_zero_video_batches(gpu, N):
    """video = None at the sizes the bench and the workspace plan care about: N = 256 is BASELINE configs[2]'s
    audio-branch batch (bench leg audio_fp32_split_b256); N = 120 sizes the split-K workspace for the dense layers only,
    while the one-clip zero-video encoder's v_conv6 splits 36 ways (it must use its own arena layout: ADVICE r4)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=12, randomize=True))
    rng = np.random.default_rng(N)
    mel = rng.normal(-40, 15, (N, 80, 20)).astype(np.float32)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), None, checked=True).cpu().numpy()
    clips = spread_clips(N, k=12)
    ref = K.forward(model.layer_dict(), mel[clips], None)
    ae, re = abs_rms(got[clips], ref), rel_rms(got[clips], ref)
    print(f"split zero video N={N}: abs {ae:.3e} rel {re:.3e}")
    assert np.isfinite(got).all() and ae <= FP32_ABS and re <= FP32_REL
    assert dw.last_range_bits == 0


def test_fp32_zero_video_large_batch(gpu):
    """AVSE_F32 with video = None at N = 4096: no layer splits K at that batch, so the forward's own split-K workspace
    is empty, while the one-clip zero-video encoder's v_conv6 splits (it wrote past the arena)."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    N = 4096
    model = KerasModel.init(seed=13, randomize=True)
    rng = np.random.default_rng(4096)
    mel = rng.normal(-40, 15, (N, 80, 20)).astype(np.float32)
    dw = ops.DeviceWeights(model, "float32")
    got = ops.forward(dw, ops.to_device(mel), None).cpu().numpy()
    clips = spread_clips(N, k=8)
    ref = K.forward(model.layer_dict(), mel[clips], None)
    assert np.isfinite(got).all() and rel_rms(got[clips], ref) <= FP32_REL


def test_split_zero_video(gpu):
    """video = None (BASELINE configs[2]): the N = 1 split video encoder on the all-zero clip, broadcast."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=5, randomize=True))
    mel, _ = make_inputs(6, 44)
    ref = K.forward(model.layer_dict(), mel, None)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), None).cpu().numpy()
    assert abs_rms(got, ref) <= FP32_ABS and rel_rms(got, ref) <= FP32_REL


@pytest.mark.parametrize("T,F", [(24, 5), (24, 6)])
def test_split_other_frame_rates(gpu, T, F):
    """29.97 fps (T = 24, 5 frames) and 30 fps (T = 24, 6 frames) networks in the split dtype: the video encoder runs
    the split v_conv1 (k_conv_v1p at 5 frames, the row-run k_conv_v1s<8, 6> at 6; conv_v1r.hip) and the split stream
    kernels at both rates;
    the T = 24 audio / decoder layers run the generic split k_conv."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from conftest import synth_video
    model = db_scale(KerasModel.init(seed=2, randomize=True, audio_shape=(80, T), video_shape=(128, 128, F)))
    rng = np.random.default_rng(3)
    mel = rng.normal(-40, 15, (3, 80, T)).astype(np.float32)
    video = synth_video(rng, 3, f=F)
    ref = K.forward(model.layer_dict(), mel, video)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
    print(f"split T={T} F={F}: abs {abs_rms(got, ref):.3e} rel {rel_rms(got, ref):.3e}")
    assert abs_rms(got, ref) <= FP32_ABS and rel_rms(got, ref) <= FP32_REL


def test_split_small_activations(gpu):
    """Tiny inputs (video x 1e-4, no normaliser): activations whose lo pieces are f16 subnormals; the error stays
    within the fp32 bounds relative to the output."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=8, randomize=True)
    mel, video = make_inputs(3, 12)
    video = (video * 1e-4).astype(np.float32)
    ref = K.forward(model.layer_dict(), mel, video)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
    print(f"split tiny video: rel {rel_rms(got, ref):.3e}")
    assert rel_rms(got, ref) <= FP32_REL


@pytest.mark.parametrize("dtype", [SPLIT, "float32"])
def test_fp32_forward_is_batch_invariant(gpu, dtype):
    """The fp32-accurate forwards give every clip the same bits whatever batch it runs in: split-K plans either split
    into whole fp32 summation blocks (v_conv6: one block per split, reduced in order) or into groups fixed by K and
    Cout alone (the split dtype's dense layers), never by the batch.  600 clips at once against the same clips run
    alone (N = 1: the most split-K) and in a batch of 7."""
    from avse_amd import ops
    from avse_amd.model import KerasModel
    import bench
    N = 600
    rng = np.random.default_rng(77)
    audio_np, video_np = bench.synth(rng, N)
    mean_np = video_np.mean(axis=(0, 3)).astype(np.float32)
    std_np = video_np.std(axis=(0, 3)).astype(np.float32)
    model = KerasModel.init(seed=3, randomize=True)
    dw = ops.DeviceWeights(model, dtype)
    mel = ops.spectrogram(ops.to_device(audio_np), frames_per_slice=20).view(N, 80, 20)
    video, mean, std = ops.to_device(video_np), ops.to_device(mean_np), ops.to_device(std_np)
    full = ops.forward(dw, mel, video, mean, std).cpu().numpy()
    for c in (0, 299, 599):
        one = ops.forward(dw, mel[c:c + 1].contiguous(), video[c:c + 1].contiguous(), mean, std).cpu().numpy()
        assert np.array_equal(one.reshape(full[c].shape), full[c]), (c, float(np.abs(one.reshape(full[c].shape) - full[c]).max()))
    part = ops.forward(dw, mel[290:297].contiguous(), video[290:297].contiguous(), mean, std).cpu().numpy()
    assert np.array_equal(part, full[290:297])


@pytest.mark.parametrize("N", [3, 37])
def test_split_windowed_layers_match_kconv_and_oracle(gpu, N):
    """conv_win.hip (the split single-phase 16-tap gather layers: d_deconv4, a_conv2) against the same layers on k_conv
    (option no_win) and the float64 oracle, layer by layer: another K order over the same products (chunk-outer,
    tap-inner), so the two agree within fp32 rounding; N = 37 puts tile boundaries inside clips and tiles over two."""
    from avse_amd import _lib
    from avse_amd.model import KerasModel
    from avse_amd import ops
    model = db_scale(KerasModel.init(seed=31, randomize=True))
    mel, video = make_inputs(N, 131)
    inter = {}
    ref = K.forward(model.layer_dict(), mel, video, intermediates=inter)
    names = ["a_conv2", "d_deconv1", "d_deconv2", "d_deconv3", "d_deconv4"]
    dw = ops.DeviceWeights(model, SPLIT)
    with _lib.context().options(no_dectail=1):   # d_deconv4 materialised (the fused tail keeps it in LDS)
        got = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
        sc = scratch(dw, N, names=names)
    with _lib.context().options(no_win=1, no_dectail=1):
        got_k = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
        sck = scratch(dw, N, names=names)
    for k in names:
        print(f"{k}: window vs oracle {rel_rms(sc[k], inter[k]):.2e}, vs k_conv {rel_rms(sc[k], sck[k]):.2e}")
        assert rel_rms(sc[k], inter[k]) <= FP32_REL and rel_rms(sc[k], sck[k]) <= 1e-6, k
    ae, aek = abs_rms(got, ref), abs_rms(got_k, ref)
    print(f"output abs RMS: windowed {ae:.3e}, k_conv {aek:.3e}")
    assert ae <= FP32_ABS and rel_rms(got, got_k) <= 1e-6


@pytest.mark.parametrize("N", [1, 3, 37, 512])
def test_split_fused_tail_matches_layer_path(gpu, N):
    """conv_dects.hip (d_deconv4 -> d_deconv5 -> d_deconv6 on split pairs, one workgroup per half clip, d_deconv4's
    output in LDS) against the layer-by-layer path (option no_dectail: k_conv_win + k_conv with the fused d_deconv6 dot)
    and the float64 oracle: the same products in another summation order, so the two agree within fp32 rounding; both
    halves of every clip (the recomputed d_deconv4 row at the seam), N = 1 .. the bench batch."""
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=41, randomize=True))
    mel, video = make_inputs(N, 141)
    dw = ops.DeviceWeights(model, SPLIT)
    fused = ops.forward(dw, ops.to_device(mel), ops.to_device(video), checked=True).cpu().numpy()
    assert dw.last_range_bits == 0
    with _lib.context().options(no_dectail=1):
        layer = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
    clips = spread_clips(N, k=6)
    ref = K.forward(model.layer_dict(), mel[clips], video[clips])
    ae, ael = abs_rms(fused[clips], ref), abs_rms(layer[clips], ref)
    d = rel_rms(fused, layer)
    print(f"N={N}: fused tail vs layer path rel {d:.2e}; abs RMS vs oracle fused {ae:.3e} layer {ael:.3e}")
    assert np.isfinite(fused).all()
    assert d <= 1e-6, d
    assert ae <= FP32_ABS and rel_rms(fused[clips], ref) <= FP32_REL
    # the seam: output rows 38..41 come from d_deconv4 rows 19 / 20, computed by both halves
    seam = rel_rms(fused[:, 36:44], layer[:, 36:44])
    assert seam <= 1e-6, seam


@pytest.mark.parametrize("N", [1, 37, 512])
def test_split_packed_v1_matches_v1s_and_oracle(gpu, N):
    """k_conv_v1p (5-frame v_conv1 with K = 128: frames 0..3 as 8-byte pixels, frame 4 scattered into row / column
    runs; conv_v1r.hip) against k_conv_v1s (K = 160 of 12-byte pixels, option no_v1p at weight load) and the float64
    oracle: the same products grouped into other 32-product MFMA sums, so the two agree within fp32 rounding; every
    tile of the 128 x 128 frames (the zero-padded borders included), one clip .. the bench batch."""
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=51, randomize=True))
    mel, video = make_inputs(N, 151)
    mean = video.mean(axis=(0, 3)).astype(np.float32)
    std = (video.std(axis=(0, 3)) + 0.1).astype(np.float32)
    names = ["v_conv1", "v_conv2"]
    dw = ops.DeviceWeights(model, SPLIT)
    with _lib.context().options(no_v1p=1):
        dw_s = ops.DeviceWeights(model, SPLIT)
    args = (ops.to_device(mel), ops.to_device(video), ops.to_device(mean), ops.to_device(std))
    clips = spread_clips(N, k=4)
    got = ops.forward(dw, *args, checked=True).cpu().numpy()
    assert dw.last_range_bits == 0
    sc = scratch(dw, N, clips, names)
    got_s = ops.forward(dw_s, *args).cpu().numpy()
    sc_s = scratch(dw_s, N, clips, names)
    inter = {}
    vn = R.video_normalize(video[clips], mean, std).astype(np.float32)
    ref = K.forward(model.layer_dict(), mel[clips], vn, intermediates=inter)
    for k in names:
        print(f"{k}: packed vs oracle {rel_rms(sc[k], inter[k]):.2e}, vs v1s {rel_rms(sc[k], sc_s[k]):.2e}")
        assert rel_rms(sc[k], inter[k]) <= FP32_REL and rel_rms(sc[k], sc_s[k]) <= 1e-6, k
    ae = abs_rms(got[clips], ref)
    print(f"N={N}: output abs RMS {ae:.3e}, packed vs v1s rel {rel_rms(got, got_s):.2e}")
    assert np.isfinite(got).all() and ae <= FP32_ABS and rel_rms(got, got_s) <= 1e-6


@pytest.mark.parametrize("N", [1, 37, 512])
def test_split_gemm_matches_kconv_and_oracle(gpu, N):
    """gemm.hip's split-pair k_gemm (v_conv6 as an implicit GEMM with the 2x2 pool, enc_dense / dec_dense1 / dec_dense2
    with split-K over whole fp32 summation blocks) against the same layers on k_conv + split-K reduce (option no_gemm)
    and the float64 oracle, layer by layer: the same products in other MFMA groupings, so the two agree within fp32
    rounding; N = 1 takes v_conv6's 36-way split, N = 512 none."""
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=61, randomize=True))
    mel, video = make_inputs(N, 161)
    names = ["concat", "enc_dense", "dec_dense1", "dec_dense2", "d_deconv1"]
    clips = spread_clips(N, k=6)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), ops.to_device(video), checked=True).cpu().numpy()
    assert dw.last_range_bits == 0
    sc = scratch(dw, N, clips, names)
    with _lib.context().options(no_gemm=1):
        got_k = ops.forward(dw, ops.to_device(mel), ops.to_device(video)).cpu().numpy()
        sck = scratch(dw, N, clips, names)
    inter = {}
    ref = K.forward(model.layer_dict(), mel[clips], video[clips], intermediates=inter)
    for k in names:
        print(f"{k}: k_gemm vs oracle {rel_rms(sc[k], inter[k]):.2e}, vs k_conv {rel_rms(sc[k], sck[k]):.2e}")
        assert rel_rms(sc[k], inter[k]) <= FP32_REL and rel_rms(sc[k], sck[k]) <= 1e-6, k
    ae = abs_rms(got[clips], ref)
    print(f"N={N}: output abs RMS {ae:.3e}, k_gemm vs k_conv rel {rel_rms(got, got_k):.2e}")
    assert np.isfinite(got).all() and ae <= FP32_ABS and rel_rms(got, got_k) <= 1e-6


@pytest.mark.parametrize("N,T", [(1, 20), (37, 20), (512, 20), (5, 24)])
def test_split_valu_aconv1_matches_kconv_and_oracle(gpu, N, T):
    """conv.hip k_aconv1_split (a_conv1 of the split dtype on the vector ALUs, fp32 FMAs straight from the audio input)
    against the split k_conv after audio_prep (option no_a1valu) and the float64 oracle: a_conv1's output and the
    forward's; T = 24 is the 29.97 fps geometry (Wo = 12)."""
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    model = db_scale(KerasModel.init(seed=71, randomize=True, audio_shape=(80, T)))
    rng = np.random.default_rng(171)
    mel = rng.normal(-40, 15, (N, 80, T)).astype(np.float32)
    names = ["a_conv1", "a_conv2"] if T == 20 else []   # (the scratch reader knows the 25 fps shapes)
    clips = spread_clips(N, k=6)
    dw = ops.DeviceWeights(model, SPLIT)
    got = ops.forward(dw, ops.to_device(mel), None, checked=True).cpu().numpy()
    assert dw.last_range_bits == 0
    sc = scratch(dw, N, clips, names)
    with _lib.context().options(no_a1valu=1):
        got_k = ops.forward(dw, ops.to_device(mel), None).cpu().numpy()
        sck = scratch(dw, N, clips, names)
    inter = {}
    ref = K.forward(model.layer_dict(), mel[clips], None, intermediates=inter)
    for k in names:
        print(f"{k}: VALU vs oracle {rel_rms(sc[k], inter[k]):.2e}, vs k_conv {rel_rms(sc[k], sck[k]):.2e}")
        assert rel_rms(sc[k], inter[k]) <= FP32_REL and rel_rms(sc[k], sck[k]) <= 1e-6, k
    ae = abs_rms(got[clips], ref)
    print(f"N={N} T={T}: output abs RMS {ae:.3e}, VALU vs k_conv rel {rel_rms(got, got_k):.2e}")
    assert np.isfinite(got).all() and ae <= FP32_ABS and rel_rms(got, got_k) <= 1e-6
