"""Empty batches through every device entry point of the ops layer: zero utterances / clips / slices give empty
outputs of the right shape and raise nothing (the C-ABI itself rejects NULL buffers, which a zero-size torch tensor
may hand it, so the ops layer returns before calling it).  numpy's reference behaviour for the same shapes: an
empty leading axis in, an empty leading axis out."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_empty_spectrogram_and_istft(gpu):
    from avse_amd import ops
    sig = torch.empty((0, 3200), dtype=torch.float32, device=gpu)
    mel = ops.spectrogram(sig)
    assert tuple(mel.shape) == (0, 80, 21)
    sliced = ops.spectrogram(sig, frames_per_slice=20)
    assert tuple(sliced.shape) == (0, 1, 80, 20)
    mel_u, stft = ops.spectrogram(torch.empty((0, 48000), dtype=torch.float32, device=gpu), frames_per_slice=20,
                                  return_stft=True)
    assert tuple(mel_u.shape) == (0, 15, 80, 20) and tuple(stft.shape) == (0, 321, 301)
    wav = ops.istft(mel_u, stft)
    assert tuple(wav.shape) == (0, 160 * 299)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_empty_forward(gpu, dtype):
    from avse_amd import ops
    from avse_amd.model import KerasModel
    dw = ops.DeviceWeights(KerasModel.init(seed=1), dtype)
    audio = torch.empty((0, 80, 20), dtype=torch.float32, device=gpu)
    video = torch.empty((0, 128, 128, 5), dtype=torch.float32, device=gpu)
    mean = torch.zeros((128, 128), dtype=torch.float32, device=gpu)
    std = torch.ones((128, 128), dtype=torch.float32, device=gpu)
    assert tuple(ops.forward(dw, audio, video).shape) == (0, 80, 20)
    assert tuple(ops.forward(dw, audio, video, mean, std).shape) == (0, 80, 20)
    assert tuple(ops.forward(dw, audio, None).shape) == (0, 80, 20)
    # a non-empty call on the same context afterwards still runs (the empty ones left no state behind)
    one = ops.forward(dw, torch.zeros((1, 80, 20), dtype=torch.float32, device=gpu),
                      torch.zeros((1, 128, 128, 5), dtype=torch.float32, device=gpu))
    assert tuple(one.shape) == (1, 80, 20) and bool(torch.isfinite(one).all())


def test_empty_video_normalize(gpu):
    from avse_amd import ops
    video = torch.empty((0, 128, 128, 5), dtype=torch.float32, device=gpu)
    mean = torch.zeros((128, 128), dtype=torch.float32, device=gpu)
    std = torch.ones((128, 128), dtype=torch.float32, device=gpu)
    assert ops.video_normalize_(video, mean, std) is video and tuple(video.shape) == (0, 128, 128, 5)
