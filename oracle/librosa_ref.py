"""numpy restatement of the librosa calls on the AVSE hot path — TEST INFRASTRUCTURE ONLY.

librosa is not vendored in /root/reference and is not listed in README.md (unpinned; the code
base dates from 2017, i.e. librosa 0.5/0.6).  Each function restates the published algorithm of
the librosa function the reference calls, at the call site cited:

  stft            <- librosa.core.stft            data_processor.py:79
  magphase        <- librosa.core.magphase        data_processor.py:80
  mel_filterbank  <- librosa.filters.mel          data_processor.py:83-89, :104-110
  amplitude_to_db <- librosa.amplitude_to_db      data_processor.py:94
  db_to_amplitude <- librosa.db_to_amplitude      data_processor.py:101
  istft           <- librosa.istft                data_processor.py:114

Version notes (documented in DESIGN.md):
  * 2017-era librosa padded with mode='reflect' (librosa >= 0.10 defaults to 'constant');
    `pad_mode` is a parameter here, default 'reflect'.
  * librosa < 0.6 conjugated the STFT ("to match DPWE phase") and its ISTFT undid it; the
    magnitude path is unaffected.  We follow the un-conjugated convention (librosa >= 0.6).
  * the STFT is evaluated in float64 and stored as complex64 (librosa's default dtype).
"""
import numpy as np


def hann_periodic(n):
    """scipy.signal.get_window('hann', n, fftbins=True) — the window librosa.stft uses."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def n_frames(n_samples, n_fft, hop_length):
    """Centred-STFT frame count: 1 + (L + 2*(n_fft//2) - n_fft) // hop."""
    return 1 + (n_samples + 2 * (n_fft // 2) - n_fft) // hop_length


def stft(y, n_fft, hop_length, pad_mode="reflect"):
    """librosa.core.stft(y, n_fft, hop_length), window='hann', center=True, dtype=complex64."""
    y = np.asarray(y)
    win = hann_periodic(n_fft)
    yp = np.pad(y.astype(np.float64), n_fft // 2, mode=pad_mode)
    T = 1 + (len(yp) - n_fft) // hop_length
    idx = np.arange(n_fft)[:, None] + hop_length * np.arange(T)[None, :]
    frames = yp[idx]
    return np.fft.rfft(win[:, None] * frames, axis=0).astype(np.complex64)


def magphase(D):
    mag = np.abs(D)
    phase = np.exp(1.0j * np.angle(D))
    return mag, phase


# --- Slaney mel scale (htk=False), librosa.core.time_frequency ---
_F_SP = 200.0 / 3
_MIN_LOG_HZ = 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = np.log(6.4) / 27.0


def hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    mels = f / _F_SP
    return np.where(f >= _MIN_LOG_HZ,
                    _MIN_LOG_MEL + np.log(np.maximum(f, _MIN_LOG_HZ) / _MIN_LOG_HZ) / _LOGSTEP, mels)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f = _F_SP * m
    return np.where(m >= _MIN_LOG_MEL, _MIN_LOG_HZ * np.exp(_LOGSTEP * (m - _MIN_LOG_MEL)), f)


def mel_filterbank(sr, n_fft, n_mels=80, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm=1) (Slaney, area-normalised)."""
    if fmax is None:
        fmax = sr / 2.0
    n_bins = 1 + n_fft // 2
    weights = np.zeros((n_mels, n_bins), dtype=np.float64)
    fftfreqs = np.linspace(0, float(sr) / 2, n_bins, endpoint=True)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, None]
    return weights


def amplitude_to_db(S, ref=1.0, amin=1e-5, top_db=80.0):
    """librosa.amplitude_to_db: power_to_db(|S|^2, ref^2, amin^2, top_db), max over the WHOLE array."""
    power = np.square(np.abs(S))
    log_spec = 10.0 * np.log10(np.maximum(amin ** 2, power))
    log_spec -= 10.0 * np.log10(np.maximum(amin ** 2, ref ** 2))
    if top_db is not None:
        log_spec = np.maximum(log_spec, log_spec.max() - top_db)
    return log_spec


def db_to_amplitude(S_db, ref=1.0):
    return (ref ** 2 * np.power(10.0, 0.1 * S_db)) ** 0.5


def window_sumsquare(n_frames_, hop_length, n_fft, dtype=np.float32):
    win_sq = hann_periodic(n_fft) ** 2
    n = n_fft + hop_length * (n_frames_ - 1)
    x = np.zeros(n, dtype=dtype)
    for i in range(n_frames_):
        s = i * hop_length
        x[s:min(n, s + n_fft)] += win_sq[:max(0, min(n_fft, n - s))]
    return x


def istft(stft_matrix, hop_length, dtype=np.float32):
    """librosa.istft(stft_matrix, hop_length), window='hann', center=True (librosa 0.6 algorithm)."""
    n_fft = 2 * (stft_matrix.shape[0] - 1)
    win = hann_periodic(n_fft)
    T = stft_matrix.shape[1]
    n = n_fft + hop_length * (T - 1)
    y = np.zeros(n, dtype=dtype)
    frames = np.fft.irfft(stft_matrix, n=n_fft, axis=0)   # == ifft(conj-symmetric spec).real
    for i in range(T):
        s = i * hop_length
        y[s:s + n_fft] = y[s:s + n_fft] + win * frames[:, i]
    wss = window_sumsquare(T, hop_length, n_fft, dtype=dtype)
    nz = wss > np.finfo(wss.dtype).tiny
    y[nz] /= wss[nz]
    return y[n_fft // 2: -(n_fft // 2)]


# ----------------------------------------------------------------------------------------------
# data_processor.py restatements
# ----------------------------------------------------------------------------------------------

def signal_to_spectrogram(signal, sample_rate, n_fft, hop_length, mel=True, db=True, pad_mode="reflect"):
    """data_processor.py:77-96 (signal = channel 0 of the AudioSignal, :78)."""
    D = stft(signal, n_fft=n_fft, hop_length=hop_length, pad_mode=pad_mode)
    magnitude, phase = magphase(D)
    if mel:
        fb = mel_filterbank(sample_rate, n_fft, n_mels=80, fmin=0, fmax=8000)
        magnitude = np.dot(fb, magnitude)
    if db:
        magnitude = amplitude_to_db(magnitude)
    return magnitude, phase


def frame_geometry(sample_rate, slice_duration_ms, n_video_slices, video_frame_rate):
    """Integer geometry of data_processor.py:36-50 (bit-exact)."""
    samples_per_slice = int((float(slice_duration_ms) / 1000) * sample_rate)
    signal_length = samples_per_slice * n_video_slices
    n_fft = int(float(sample_rate) / video_frame_rate)
    hop_length = int(n_fft / 4)
    spf = int(samples_per_slice / hop_length)
    T = n_frames(signal_length, n_fft, hop_length)
    n_slices = int(T / spf)
    return dict(samples_per_slice=samples_per_slice, signal_length=signal_length, n_fft=n_fft,
                hop_length=hop_length, spectrogram_samples_per_slice=spf, n_frames=T, n_slices=n_slices)


def fit_length(signal, signal_length):
    """pad_with_zeros / truncate (data_processor.py:39-42)."""
    signal = np.asarray(signal)
    if len(signal) < signal_length:
        return np.concatenate([signal, np.zeros(signal_length - len(signal), dtype=signal.dtype)])
    return signal[:signal_length]


def preprocess_audio_signal(signal, sample_rate, slice_duration_ms, n_video_slices, video_frame_rate,
                            pad_mode="reflect"):
    """data_processor.py:35-57 -> [n_slices, 80, spf]."""
    g = frame_geometry(sample_rate, slice_duration_ms, n_video_slices, video_frame_rate)
    sig = fit_length(signal, g["signal_length"])
    mel_db, _ = signal_to_spectrogram(sig, sample_rate, g["n_fft"], g["hop_length"], pad_mode=pad_mode)
    spf = g["spectrogram_samples_per_slice"]
    n = int(mel_db.shape[1] / spf)
    return np.stack([mel_db[:, i * spf:(i + 1) * spf] for i in range(n)])


def reconstruct_signal_from_spectrogram(magnitude, phase, sample_rate, n_fft, hop_length):
    """data_processor.py:99-116 (mel=True, db=True)."""
    magnitude = db_to_amplitude(magnitude)
    fb = mel_filterbank(sample_rate, n_fft, n_mels=80, fmin=0, fmax=8000)
    magnitude = np.dot(np.linalg.pinv(fb), magnitude)
    return istft(magnitude * phase, hop_length=hop_length)


def reconstruct_speech_signal(mixed_signal, sample_rate, speech_spectrograms, video_frame_rate,
                              pad_mode="reflect"):
    """data_processor.py:60-74."""
    n_fft = int(float(sample_rate) / video_frame_rate)
    hop_length = int(n_fft / 4)
    _, original_phase = signal_to_spectrogram(mixed_signal, sample_rate, n_fft, hop_length, pad_mode=pad_mode)
    speech = np.concatenate(list(speech_spectrograms), axis=1)
    L = min(speech.shape[1], original_phase.shape[1])
    return reconstruct_signal_from_spectrogram(speech[:, :L], original_phase[:, :L], sample_rate, n_fft, hop_length)


def video_normalizer_fit(video_samples):
    """VideoNormalizer.__init__ (data_processor.py:203-206): mean/std over axes (0, 3)."""
    return np.mean(video_samples, axis=(0, 3)), np.std(video_samples, axis=(0, 3))


def video_normalize(video_samples, mean_image, std_image):
    """VideoNormalizer.normalize (data_processor.py:208-212), out of place."""
    return (video_samples - mean_image[None, :, :, None]) / std_image[None, :, :, None]
