"""Reference-shaped audio front end (mirrors /root/reference/data_processor.py), computed by libavse.

Same function names, arguments, return shapes and in-place side effects as the reference; the
arithmetic runs in the HIP kernels behind include/avse.h.  Inputs may be numpy (returned as numpy,
as in the reference) or ROCm tensors (returned as tensors).
"""
import numpy as np
import torch

from . import ops
from .audio_io import AudioSignal

N_MELS = 80          # data_processor.py:86
MEL_FMIN = 0         # data_processor.py:87
MEL_FMAX = 8000      # data_processor.py:88


def frame_geometry(sample_rate, slice_duration_ms, n_video_slices, video_frame_rate):
    """Integer geometry of preprocess_audio_signal (data_processor.py:36-50), bit-exact."""
    samples_per_slice = int((float(slice_duration_ms) / 1000) * sample_rate)
    signal_length = samples_per_slice * n_video_slices
    n_fft = int(float(sample_rate) / video_frame_rate)
    hop_length = int(n_fft / 4)
    spf = int(samples_per_slice / hop_length)
    T = ops.n_frames(signal_length, hop_length, n_fft)
    return dict(samples_per_slice=samples_per_slice, signal_length=signal_length, n_fft=n_fft,
                hop_length=hop_length, spectrogram_samples_per_slice=spf, n_frames=T, n_slices=int(T / spf))


def _channel0(audio_signal):
    return audio_signal.get_data(channel_index=0)


def signal_to_spectrogram(audio_signal, n_fft, hop_length, mel=True, db=True):
    """data_processor.py:77-96 -> (mel-dB [80, T], phase [n_fft//2+1, T] complex64), as numpy."""
    if not (mel and db):
        raise NotImplementedError("the reference calls signal_to_spectrogram with mel=True, db=True only "
                                  "(data_processor.py:47, :64, :73)")
    sig = ops.to_device(np.asarray(_channel0(audio_signal))[None, :])
    mel_db, D = ops.spectrogram(sig, sample_rate=audio_signal.get_sample_rate(), n_fft=n_fft, hop_length=hop_length,
                                n_mels=N_MELS, fmin=MEL_FMIN, fmax=MEL_FMAX, return_stft=True)
    mag = D.abs()
    phase = torch.where(mag > 0, D / mag.clamp_min(1e-38), torch.ones_like(D))   # exp(1j * angle(D))
    return mel_db[0].cpu().numpy(), phase[0].cpu().numpy()


def preprocess_audio_signal(audio_signal, slice_duration_ms, n_video_slices, video_frame_rate):
    """data_processor.py:35-57: pad/truncate the signal IN PLACE, STFT the whole utterance, cut
    into [n_slices, 80, spf] slices (trailing frames dropped; the top_db max still sees them)."""
    g = frame_geometry(audio_signal.get_sample_rate(), slice_duration_ms, n_video_slices, video_frame_rate)
    if audio_signal.get_number_of_samples() < g["signal_length"]:
        audio_signal.pad_with_zeros(g["signal_length"])
    else:
        audio_signal.truncate(g["signal_length"])
    sig = ops.to_device(np.asarray(_channel0(audio_signal))[None, :])
    out = ops.spectrogram(sig, sample_rate=audio_signal.get_sample_rate(), n_fft=g["n_fft"],
                          hop_length=g["hop_length"], n_mels=N_MELS, fmin=MEL_FMIN, fmax=MEL_FMAX,
                          frames_per_slice=g["spectrogram_samples_per_slice"])
    return out[0].cpu().numpy()


def preprocess_audio_batch(signals, sample_rate, slice_duration_ms, n_video_slices, video_frame_rate):
    """Batched preprocess_audio_signal for equal-length device signals [U, L] -> [U, n_slices, 80, spf]
    (device tensor).  Each row is padded/truncated to the slice geometry first."""
    g = frame_geometry(sample_rate, slice_duration_ms, n_video_slices, video_frame_rate)
    L = g["signal_length"]
    if signals.shape[1] < L:
        signals = torch.nn.functional.pad(signals, (0, L - signals.shape[1]))
    signals = signals[:, :L].contiguous()
    return ops.spectrogram(signals, sample_rate=sample_rate, n_fft=g["n_fft"], hop_length=g["hop_length"],
                           n_mels=N_MELS, fmin=MEL_FMIN, fmax=MEL_FMAX,
                           frames_per_slice=g["spectrogram_samples_per_slice"])


def reconstruct_speech_signal(mixed_signal, speech_spectrograms, video_frame_rate):
    """data_processor.py:60-74: phase of the mixture's STFT + predicted speech mel-dB slices
    [n_slices, 80, spf] -> AudioSignal (K1 for the phase, K6 for the inverse)."""
    sr = mixed_signal.get_sample_rate()
    n_fft = int(float(sr) / video_frame_rate)
    hop_length = int(n_fft / 4)
    sig = ops.to_device(np.asarray(_channel0(mixed_signal))[None, :])
    _, D = ops.spectrogram(sig, sample_rate=sr, n_fft=n_fft, hop_length=hop_length, n_mels=N_MELS, fmin=MEL_FMIN,
                           fmax=MEL_FMAX, return_stft=True)
    spec = ops.to_device(speech_spectrograms, sig.device)
    if spec.dim() == 2:                      # predict() squeezes a single slice to [80, spf]
        spec = spec[None]
    y = ops.istft(spec[None].contiguous(), D, sample_rate=sr, n_fft=n_fft, hop_length=hop_length, n_mels=N_MELS,
                  fmin=MEL_FMIN, fmax=MEL_FMAX)
    return AudioSignal(y[0].cpu().numpy(), sr)


def reconstruct_signal_from_spectrogram(magnitude, phase, sample_rate, n_fft, hop_length, mel=True, db=True):
    """data_processor.py:99-116 for mel-dB `magnitude` [80, T] and unit `phase` [n_fft//2+1, T]."""
    if not (mel and db):
        raise NotImplementedError("the reference calls it with mel=True, db=True only (data_processor.py:72-74)")
    m = ops.to_device(magnitude)[None].contiguous()
    ph = torch.from_numpy(np.ascontiguousarray(phase, dtype=np.complex64)).to(m.device)[None]
    y = ops.istft(m, ph, sample_rate=sample_rate, n_fft=n_fft, hop_length=hop_length, n_mels=N_MELS, fmin=MEL_FMIN,
                  fmax=MEL_FMAX)
    return AudioSignal(y[0].cpu().numpy(), sample_rate)


class VideoNormalizer(object):
    """data_processor.py:201-212.  Statistics are fitted over axes (0, 3) like the reference
    (training-time, host numpy float32); normalize() runs in libavse and mutates its argument."""

    def __init__(self, video_samples):
        # video_samples: slices x height x width x frames_per_slice
        v = video_samples.cpu().numpy() if isinstance(video_samples, torch.Tensor) else video_samples
        self.__mean_image = np.mean(v, axis=(0, 3))
        self.__std_image = np.std(v, axis=(0, 3))

    @property
    def mean_image(self):
        return self.__mean_image

    @property
    def std_image(self):
        return self.__std_image

    @classmethod
    def from_stats(cls, mean_image, std_image):
        obj = cls.__new__(cls)
        obj.__mean_image = np.asarray(mean_image, np.float32)
        obj.__std_image = np.asarray(std_image, np.float32)
        return obj

    def save(self, path):
        """The fitted images as .npz (the reference pickles the object: speech_enhancer.py:48-49)."""
        with open(path, "wb") as fd:
            np.savez(fd, mean_image=self.__mean_image, std_image=self.__std_image)

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            return cls.from_stats(z["mean_image"], z["std_image"])

    def device_stats(self, device=None):
        return ops.to_device(self.__mean_image, device), ops.to_device(self.__std_image, device)

    def normalize(self, video_samples):
        """In place, like data_processor.py:208-212."""
        if isinstance(video_samples, torch.Tensor) and video_samples.is_cuda:
            m, s = self.device_stats(video_samples.device)
            ops.video_normalize_(video_samples, m, s)
            return
        if not (isinstance(video_samples, np.ndarray) and video_samples.dtype == np.float32):
            raise TypeError("normalize expects a float32 numpy array or a ROCm tensor (it works in place)")
        v = ops.to_device(video_samples)
        m, s = self.device_stats(v.device)
        ops.video_normalize_(v, m, s)
        video_samples[...] = v.cpu().numpy()
