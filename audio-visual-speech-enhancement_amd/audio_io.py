"""Minimal stand-in for the un-vendored `mediaio.audio_io` (AudioSignal, AudioMixer) the reference
imports at /root/reference/data_processor.py:8.  Only the methods the reference calls are provided:

  AudioSignal(data, sample_rate), .from_wav_file, .save_to_wav_file, .get_data(channel_index),
  .get_sample_rate, .get_number_of_samples, .pad_with_zeros, .truncate (in place,
  data_processor.py:39-42), .amplify_by_factor, AudioSignal.concat (data_processor.py:126)
  AudioMixer.snr_factor, AudioMixer.mix (data_processor.py:130-133)

This is host-side file plumbing (out of the hot path).
"""
import numpy as np


class AudioSignal:
    def __init__(self, data, sample_rate):
        data = np.asarray(data)
        self._data = data if data.ndim == 2 else data[:, None]     # [n_samples, n_channels]
        self._sample_rate = int(sample_rate)

    @classmethod
    def from_wav_file(cls, path):
        from scipy.io import wavfile
        sr, data = wavfile.read(path)
        return cls(data, sr)

    def save_to_wav_file(self, path, dtype=np.int16):
        from scipy.io import wavfile
        data = self._data
        if np.issubdtype(dtype, np.integer) and not np.issubdtype(data.dtype, np.integer):
            info = np.iinfo(dtype)
            data = np.clip(np.round(data), info.min, info.max)
        wavfile.write(path, self._sample_rate, data.astype(dtype).squeeze())

    def get_data(self, channel_index=None):
        if channel_index is None:
            return self._data
        return self._data[:, channel_index]

    def get_sample_rate(self):
        return self._sample_rate

    def get_number_of_samples(self):
        return self._data.shape[0]

    def get_number_of_channels(self):
        return self._data.shape[1]

    def pad_with_zeros(self, new_length):
        if self._data.shape[0] < new_length:
            pad = np.zeros((new_length - self._data.shape[0], self._data.shape[1]), dtype=self._data.dtype)
            self._data = np.concatenate([self._data, pad], axis=0)

    def truncate(self, new_length):
        self._data = self._data[:new_length]

    def amplify_by_factor(self, factor):
        self._data = self._data.astype(np.float64) * factor

    @staticmethod
    def concat(signals):
        sr = signals[0].get_sample_rate()
        return AudioSignal(np.concatenate([s.get_data() for s in signals], axis=0), sr)


class AudioMixer:
    @staticmethod
    def snr_factor(signal, noise, snr_db):
        s = np.mean(signal.get_data().astype(np.float64) ** 2)
        n = np.mean(noise.get_data().astype(np.float64) ** 2)
        if n == 0:
            return 0.0
        return float(np.sqrt(s / (n * 10.0 ** (snr_db / 10.0))))

    @staticmethod
    def mix(signals, mixing_weights=None):
        if mixing_weights is None:
            mixing_weights = [1] * len(signals)
        sr = signals[0].get_sample_rate()
        out = sum(w * s.get_data().astype(np.float64) for s, w in zip(signals, mixing_weights))
        return AudioSignal(out, sr)
