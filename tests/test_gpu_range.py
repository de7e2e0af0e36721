"""AVSE_F32_SPLIT range safety (include/avse.h: the range guard and the per-layer activation exponents).

The split dtype carries activations as f16 pairs h + l: |x| >= 65520 overflows h, and a layer whose activations are
all tiny puts its lo pieces in the f16 subnormal range.  The float32 Keras reference (/root/reference/network.py:208-212)
has neither limit, so:
  * every kernel that stores a pair (or splits an fp32 input) reports an out-of-range value into a range guard, and
    avse_forward_checked recomputes such a batch on the exact-fp32 kernels (never inf / NaN where fp32 is finite) or
    fails with AVSE_ERR_RANGE;
  * each layer's pairs carry x 2^e_L with e_L from its BatchNormalization parameters, so a model whose BN puts a layer's
    activations far from O(1) keeps ~22 bits (tiny) or its headroom (huge).
The models here compute the same function as an ordinary random-init model: a layer's BN gamma / beta are scaled by
2^k and the next layer's kernel by 2^-k (powers of two: exact, and they commute with LeakyReLU), or a kernel is scaled
so that the BN statistics no longer describe the activations (the guard's case).
"""
import numpy as np
import pytest

from oracle import keras_ref as K
from test_gpu_forward import FP32_ABS, FP32_REL, abs_rms, db_scale, make_inputs, rel_rms

pytestmark = pytest.mark.gpu

SPLIT = "float32_split"


def _run(model, mel, video, dtype=SPLIT, checked=True, **kw):
    """The checked forward (avse_forward_checked): the guard bits are read before it returns."""
    from avse_amd import ops
    dw = ops.DeviceWeights(model, dtype)
    v = None if video is None else ops.to_device(video)
    return ops.forward(dw, ops.to_device(mel), v, checked=checked, **kw).cpu().numpy(), dw


def _rescaled(model, layer, nxt, k):
    """layer's BN gamma, beta x 2^k and nxt's kernel x 2^-k: the same network function, layer's activations x 2^k"""
    t = model.tensors
    for p in ("gamma", "beta"):
        t[f"{layer}_bn/{p}"] = (t[f"{layer}_bn/{p}"] * np.float32(2.0 ** k)).astype(np.float32)
    t[f"{nxt}/kernel"] = (t[f"{nxt}/kernel"] * np.float32(2.0 ** -k)).astype(np.float32)
    return model


def test_overflow_is_recomputed_on_exact_fp32(gpu):
    """v_conv2's kernel x 3000 (BN identity statistics unchanged): its activations reach ~1e5 — past the f16 range, not
    predicted by the BN parameters.  The checked forward reports v_conv2 and returns the exact-fp32 forward bit for bit;
    the error mode raises; an unchecked forward leaves the bits for avse_range_status."""
    import warnings
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=6, randomize=True)
    model.tensors["v_conv2/kernel"] = (model.tensors["v_conv2/kernel"] * np.float32(3000.0)).astype(np.float32)
    mel, video = make_inputs(3, 61)
    inter = {}
    ref = K.forward(model.layer_dict(), mel, video, intermediates=inter)
    print(f"v_conv2 activation max {np.abs(inter['v_conv2']).max():.3g}")
    assert np.abs(inter["v_conv2"]).max() > 65520.0
    ctx = _lib.context()
    ctx.range_status()   # clear
    with pytest.warns(RuntimeWarning, match="v_conv2"):
        got, dw = _run(model, mel, video)
    assert dw.last_range_bits >> 6 & 1, hex(dw.last_range_bits)
    f32, _ = _run(model, mel, video, "float32")
    assert np.isfinite(got).all()
    assert np.array_equal(got, f32)
    assert rel_rms(got, ref) <= FP32_REL
    with pytest.raises(_lib.RangeError):
        ops.forward(dw, ops.to_device(mel), ops.to_device(video), checked=True, on_range="error")
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        ops.forward(dw, ops.to_device(mel), ops.to_device(video), checked=False)
    bits = ctx.range_status()
    assert bits >> 6 & 1 and _lib.range_bit_names(bits)[0] == "v_conv2", hex(bits)
    assert ctx.range_status() == 0    # read and cleared


@pytest.mark.parametrize("which", ["audio", "video"])
def test_input_overflow_is_recomputed(gpu, which):
    """Network inputs past the f16 range (split on load: a_conv1's slab store, v_conv1's window loader)."""
    from avse_amd.model import KerasModel
    model = KerasModel.init(seed=7, randomize=True)
    mel, video = make_inputs(2, 62)
    if which == "audio":
        mel = mel.copy()
        mel[1, 3, 4] = 1e5
    else:
        video = (video * 1000.0).astype(np.float32)
    ref = K.forward(model.layer_dict(), mel, video)
    with pytest.warns(RuntimeWarning):
        got, dw = _run(model, mel, video)
    bit = 24 if which == "audio" else 25
    assert dw.last_range_bits >> bit & 1, hex(dw.last_range_bits)
    f32, _ = _run(model, mel, video, "float32")
    assert np.array_equal(got, f32) and np.isfinite(got).all()
    assert rel_rms(got, ref) <= FP32_REL


def test_zero_video_embedding_overflow_reported_every_call(gpu):
    """video = None: the all-zero-video embedding is computed once per weights object and cached; when its computation
    overflowed, every later forward that broadcasts it reports (and recomputes) too."""
    from avse_amd.model import KerasModel
    from avse_amd import ops
    model = KerasModel.init(seed=8, randomize=True)
    model.tensors["v_conv6/kernel"] = (model.tensors["v_conv6/kernel"] * np.float32(1e6)).astype(np.float32)
    mel, _ = make_inputs(4, 63)
    ref = K.forward(model.layer_dict(), mel, None)
    dw = ops.DeviceWeights(model, SPLIT)
    f32 = ops.forward(ops.DeviceWeights(model, "float32"), ops.to_device(mel), None).cpu().numpy()
    for _ in range(2):
        with pytest.warns(RuntimeWarning, match="v_conv6"):
            got = ops.forward(dw, ops.to_device(mel), None, checked=True).cpu().numpy()
        assert dw.last_range_bits >> 10 & 1
        assert np.array_equal(got, f32)
    assert rel_rms(got, ref) <= FP32_REL


@pytest.mark.parametrize("layer,nxt", [("v_conv3", "v_conv4"), ("a_conv2", "a_conv3"), ("d_deconv3", "d_deconv4"),
                                       ("enc_dense", "dec_dense1"), ("a_conv1", "a_conv2"), ("v_conv1", "v_conv2")])
def test_tiny_activations_keep_fp32_accuracy(gpu, layer, nxt):
    """layer's activations x 2^-14 (BN gamma / beta scaled, nxt's kernel compensating): without exponents its pairs' lo
    pieces (and some hi pieces) are f16 subnormals; with them the layer stores x 2^16 and the forward is as accurate as
    on the unscaled model (same function, same oracle output)."""
    from avse_amd import _lib
    from avse_amd.model import KerasModel
    base = db_scale(KerasModel.init(seed=9, randomize=True))
    model = _rescaled(db_scale(KerasModel.init(seed=9, randomize=True)), layer, nxt, -14)
    mel, video = make_inputs(3, 64)
    ref = K.forward(model.layer_dict(), mel, video)
    got_base, _ = _run(base, mel, video)
    got, dw = _run(model, mel, video)
    e = dw.act_exponents()
    assert e[layer] >= 14 and all(v == 0 for k, v in e.items() if k != layer), e
    assert dw.last_range_bits == 0
    with _lib.context().options(no_act_scale=1):
        got_noexp, dw0 = _run(model, mel, video)
    assert all(v == 0 for v in dw0.act_exponents().values())
    f32, _ = _run(model, mel, video, "float32")
    ae, ae0, ae32, aeb = abs_rms(got, ref), abs_rms(got_noexp, ref), abs_rms(f32, ref), abs_rms(got_base, ref)
    print(f"{layer} x 2^-14: split abs RMS {ae:.3e} (unscaled model {aeb:.3e}), without exponents {ae0:.3e}, "
          f"exact fp32 {ae32:.3e}")
    assert ae <= FP32_ABS and rel_rms(got, ref) <= FP32_REL
    assert ae <= 1.5 * aeb + 1e-6          # as accurate as the same function with O(1) activations
    assert ae0 > 3 * ae                    # the subnormal lo pieces cost accuracy without the exponent


@pytest.mark.parametrize("layer,nxt", [("v_conv2", "v_conv3"), ("dec_dense1", "dec_dense2"), ("d_deconv2", "d_deconv3"),
                                       ("d_deconv4", "d_deconv5"), ("a_conv1", "a_conv2"), ("v_conv1", "v_conv2"),
                                       ("enc_dense", "dec_dense1")])
def test_huge_activations_keep_headroom(gpu, layer, nxt):
    """layer's activations x 2^14 (~1e5 .. 1e6): with exponents the layer stores x 2^-14 .. and no pair overflows; without
    them the range guard fires and the batch is recomputed on the exact-fp32 kernels."""
    import warnings
    from avse_amd import _lib
    from avse_amd.model import KerasModel
    model = _rescaled(db_scale(KerasModel.init(seed=10, randomize=True)), layer, nxt, 14)
    mel, video = make_inputs(3, 65)
    inter = {}
    ref = K.forward(model.layer_dict(), mel, video, intermediates=inter)
    assert np.abs(inter[layer]).max() > 65520.0
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        got, dw = _run(model, mel, video)
    e = dw.act_exponents()
    assert e[layer] < 0 and dw.last_range_bits == 0, (e, hex(dw.last_range_bits))
    ae = abs_rms(got, ref)
    f32, _ = _run(model, mel, video, "float32")
    print(f"{layer} x 2^14: exponent {e[layer]}, split abs RMS {ae:.3e}, exact fp32 {abs_rms(f32, ref):.3e}")
    assert ae <= FP32_ABS and rel_rms(got, ref) <= FP32_REL
    with _lib.context().options(no_act_scale=1):
        with pytest.warns(RuntimeWarning):
            got0, dw0 = _run(model, mel, video)
    assert dw0.last_range_bits and np.array_equal(got0, f32)


def test_trained_model_split_parity(gpu):
    """Weights from this build's own training loop (fit.py over csrc/train.hip: moving statistics, gamma / beta and
    kernels moved by Adam), the output layer set to dB scale: the split forward within the north star's 1e-4 absolute
    RMS of the float64 oracle and no worse than 1.5x the exact-fp32 path."""
    import torch
    from avse_amd import fit as F
    from avse_amd.model import KerasModel
    from conftest import synth_video
    rng = np.random.default_rng(70)
    n, nv = 64, 16
    speech = rng.normal(-40, 12, (n + nv, 80, 20)).astype(np.float32)
    mixed = (speech + rng.normal(0, 6, speech.shape)).astype(np.float32)
    video = synth_video(rng, n + nv)
    video = ((video - 127.5) / 74.0).astype(np.float32)
    model = KerasModel.init(seed=11)
    trained, hist = F.fit(model, (mixed[:n], video[:n], speech[:n]), (mixed[n:], video[n:], speech[n:]), epochs=6,
                          lr=2e-3, verbose=0)
    assert hist[-1]["loss"] < hist[0]["loss"]
    t = trained.tensors
    moved = np.abs(t["v_conv3_bn/moving_mean"]).max()
    assert moved > 0, "moving statistics not updated"
    mel_t, vid_t = mixed[n:n + 6], video[n:n + 6]
    # a few epochs do not reach the target scale: the output layer (network.py:133) is set to map the trained
    # network's output to dB scale (std 10 dB about -40 dB, as db_scale does for random-init models)
    raw = K.forward(trained.layer_dict(), mel_t, vid_t)
    db_scale(trained, gain=10.0 / float(np.std(raw)))
    ref = K.forward(trained.layer_dict(), mel_t, vid_t)
    got, dw = _run(trained, mel_t, vid_t)
    f32, _ = _run(trained, mel_t, vid_t, "float32")
    ae, ae32 = abs_rms(got, ref), abs_rms(f32, ref)
    print(f"trained model: exponents {dw.act_exponents()}, split abs RMS {ae:.3e}, exact fp32 {ae32:.3e}, output RMS "
          f"{np.sqrt(np.mean(ref ** 2)):.3g}")
    assert dw.last_range_bits == 0
    assert ae <= FP32_ABS and ae <= 1.5 * ae32 + 1e-6
    torch.cuda.synchronize()


def test_range_pipeline_recomputes_flagged_batches(gpu):
    """ops.RangePipeline (avse_range_snapshot): unchecked forwards queued back to back, each batch's guard read one batch
    later; the flagged batches (the overflowing model) are recomputed on exact fp32 into their own outputs, the clean
    ones (the same model's weights at O(1) scale) are not."""
    from avse_amd import _lib, ops
    from avse_amd.model import KerasModel
    bad = KerasModel.init(seed=6, randomize=True)
    bad.tensors["v_conv2/kernel"] = (bad.tensors["v_conv2/kernel"] * np.float32(3000.0)).astype(np.float32)
    good = KerasModel.init(seed=6, randomize=True)
    mel, video = make_inputs(3, 66)
    m, v = ops.to_device(mel), ops.to_device(video)
    dws = {"bad": ops.DeviceWeights(bad, SPLIT), "good": ops.DeviceWeights(good, SPLIT)}
    ref32 = {k: ops.forward(ops.DeviceWeights(x, "float32"), m, v).cpu().numpy() for k, x in (("bad", bad), ("good", good))}
    ctx = _lib.context()
    ctx.range_status()
    pipe = ops.RangePipeline(ctx)
    outs = {}
    for name in ("good", "bad", "good", "bad"):
        out = outs.setdefault(name, [])
        o = ops.forward(dws[name], m, v, checked=False)
        out.append(o)
        pipe.submit(lambda dw=dws[name], o=o: ops.forward(dw, m, v, out=o, checked=True))
    bits = pipe.drain()
    assert bits >> 6 & 1 and pipe.recomputed == 2, (hex(bits), pipe.recomputed)
    for o in outs["bad"]:
        assert np.array_equal(o.cpu().numpy(), ref32["bad"])
    ref = K.forward(good.layer_dict(), mel, video)
    for o in outs["good"]:
        assert rel_rms(o.cpu().numpy(), ref) <= FP32_REL
