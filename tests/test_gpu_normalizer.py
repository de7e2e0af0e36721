"""VideoNormalizer (data_processor.py:201-212) on the device: the reference's IN-PLACE normalize, not only the copy
fused into v_conv1's loader.

The reference loops `video_samples[slice, :, :, frame] = (video_samples[slice, :, :, frame] - mean) / std` in numpy
float32 (data_processor.py:208-212) after fitting mean / std over axes (0, 3) (:205-206).  avse_video_normalize does
one float32 subtract and one correctly rounded float32 divide per element, so the result is BIT-EXACT against that
loop (asserted with array_equal), for numpy arrays (round trip through the device, written back in place) and for
device tensors (in place on the device).
"""
import numpy as np
import pytest
import torch

from conftest import synth_video

pytestmark = pytest.mark.gpu


def reference_normalize(video, mean, std):
    """data_processor.py:208-212, restated loop for loop (float32 numpy, in place on a copy)."""
    v = np.array(video, dtype=np.float32, copy=True)
    for s in range(v.shape[0]):
        for f in range(v.shape[3]):
            v[s, :, :, f] -= mean
            v[s, :, :, f] /= std
    return v


@pytest.mark.parametrize("S,F", [(1, 5), (7, 5), (3, 6)])   # F = 6: 30-fps slices (data_processor.py:24)
def test_normalize_numpy_in_place_is_bit_exact(gpu, S, F):
    from avse_amd.data_processor import VideoNormalizer
    rng = np.random.default_rng(S * 10 + F)
    video = synth_video(rng, S, f=F)
    norm = VideoNormalizer(video)
    # fitted like the reference: np.mean / np.std over axes (0, 3), float32 (data_processor.py:205-206)
    np.testing.assert_array_equal(norm.mean_image, np.mean(video, axis=(0, 3)))
    np.testing.assert_array_equal(norm.std_image, np.std(video, axis=(0, 3)))
    expect = reference_normalize(video, norm.mean_image, norm.std_image)
    arr = video.copy()
    ret = norm.normalize(arr)
    assert ret is None                       # like the reference: mutates its argument, returns nothing
    np.testing.assert_array_equal(arr, expect)
    assert not np.array_equal(arr, video)


def test_normalize_device_tensor_in_place(gpu):
    from avse_amd.data_processor import VideoNormalizer
    rng = np.random.default_rng(3)
    video = synth_video(rng, 9)
    norm = VideoNormalizer(video)
    t = torch.from_numpy(video.copy()).to(gpu)
    ptr = t.data_ptr()
    norm.normalize(t)
    assert t.data_ptr() == ptr
    np.testing.assert_array_equal(t.cpu().numpy(), reference_normalize(video, norm.mean_image, norm.std_image))


def test_normalize_rejects_non_float32_arrays(gpu):
    from avse_amd.data_processor import VideoNormalizer
    video = synth_video(np.random.default_rng(0), 2)
    norm = VideoNormalizer(video)
    with pytest.raises(TypeError):
        norm.normalize(video.astype(np.float64))


def test_in_place_normalize_then_forward_equals_fused_normalizer(gpu):
    """speech_enhancer.predict normalises in place and then predicts (speech_enhancer.py:74-81); this build can also
    fuse the normaliser into the video encoder's input load.  Both orders give the same network output up to float32
    rounding (fp32 weights)."""
    from avse_amd.data_processor import VideoNormalizer
    from avse_amd.model import KerasModel
    from avse_amd.network import SpeechEnhancementNetwork
    rng = np.random.default_rng(4)
    video = synth_video(rng, 6)
    mel = rng.normal(-40, 12, (6, 80, 20)).astype(np.float32)
    norm = VideoNormalizer(video)
    net = SpeechEnhancementNetwork(KerasModel.init(seed=6, randomize=True), "float32")
    fused = net.predict(mel, video, video_normalizer=norm)
    arr = video.copy()
    norm.normalize(arr)
    in_place = net.predict(mel, arr)
    rel = np.sqrt(np.mean((fused - in_place) ** 2)) / np.sqrt(np.mean(in_place ** 2))
    assert rel <= 1e-5, rel
