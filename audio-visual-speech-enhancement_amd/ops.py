"""Device-level entry points: torch (ROCm) tensors in, torch tensors out, arithmetic in libavse.

Every function here is a thin shape/dtype check around one C-ABI call (include/avse.h) launched
on torch's current HIP stream.  Nothing computes on the CPU.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .model import KerasModel, blob_floats

DTYPES = {"float32": _lib.AVSE_F32, "fp32": _lib.AVSE_F32, "bfloat16": _lib.AVSE_BF16, "bf16": _lib.AVSE_BF16,
          # float32 accuracy from split-f16 matrix-core products (include/avse.h AVSE_F32_SPLIT)
          "float32_split": _lib.AVSE_F32_SPLIT, "fp32_split": _lib.AVSE_F32_SPLIT}


def _dev_f32(t, name, shape=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a ROCm device tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape[-len(shape):]) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected [..., {shape}]")
    return t


def n_frames(n_samples, hop, n_fft):
    """Centred STFT frame count (librosa.stft, center=True): 1 + (L + 2*(n_fft//2) - n_fft) // hop."""
    return 1 + (n_samples + 2 * (n_fft // 2) - n_fft) // hop


def spectrogram(sig, sample_rate=16000, n_fft=640, hop_length=160, n_mels=80, fmin=0.0, fmax=8000.0,
                amin=1e-5, top_db=80.0, pad_mode="reflect", frames_per_slice=0, return_stft=False, out=None):
    """K1: STFT -> mel -> dB for a batch of utterances.

    sig [U, L] float32 device tensor.  Returns mel_db [U, n_mels, T] (frames_per_slice == 0) or
    [U, n_slices, n_mels, frames_per_slice] (into `out` when given); with return_stft also the complex64 STFT
    [U, 1+n_fft//2, T].
    """
    _dev_f32(sig, "sig")
    if sig.dim() != 2:
        raise ValueError("sig must be [n_utterances, n_samples]")
    U, L = sig.shape
    T = n_frames(L, hop_length, n_fft)
    shape = (U, T // frames_per_slice, n_mels, frames_per_slice) if frames_per_slice else (U, n_mels, T)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=sig.device)
    else:
        _dev_f32(out, "out")
        if tuple(out.shape) != shape or out.device != sig.device:
            raise ValueError(f"out must be {shape} on {sig.device}")
    stft = torch.empty((U, 1 + n_fft // 2, T, 2), dtype=torch.float32, device=sig.device) if return_stft else None
    pm = {"reflect": _lib.AVSE_PAD_REFLECT, "constant": _lib.AVSE_PAD_CONSTANT}[pad_mode]
    if U == 0:   # empty batch: empty outputs (the C-ABI takes no NULL buffers, even for zero utterances)
        return (out, torch.view_as_complex(stft)) if return_stft else out
    ctx = _lib.context(sig.device)
    with torch.cuda.device(sig.device):
        _lib.check(_lib.load().avse_spectrogram(
            ctx.handle, _lib.ptr(sig), U, L, int(sample_rate), int(n_fft), int(hop_length), int(n_mels),
            float(fmin), float(fmax), float(amin), float(-1.0 if top_db is None else top_db), pm,
            int(frames_per_slice), _lib.ptr(out), _lib.ptr(stft), _lib.stream_handle(sig.device)), "avse_spectrogram")
    if return_stft:
        return out, torch.view_as_complex(stft)
    return out


def istft(mel_db, stft, sample_rate=16000, n_fft=640, hop_length=160, n_mels=80, fmin=0.0, fmax=8000.0,
          n_frames=None):
    """K6: speech mel-dB + mixture STFT -> time signal (reconstruct_signal_from_spectrogram).

    mel_db: [U, n_slices, n_mels, spf] (network output of consecutive slices) or [U, n_mels, T];
    stft: complex64 [U, n_fft//2+1, T_stft] (or its float32 [..., 2] view) from spectrogram(return_stft=True).
    Uses the first n_frames = min(T_pred, T_stft) frames (data_processor.py:68-70).
    Returns [U, hop * (n_frames - 1)] float32."""
    _dev_f32(mel_db, "mel_db")
    if stft.dtype == torch.complex64:
        stft = torch.view_as_real(stft)
    _dev_f32(stft, "stft")
    if mel_db.dim() == 4:
        U, ns, nm, spf = mel_db.shape
        T_pred = ns * spf
    else:
        U, nm, T_pred = mel_db.shape
        spf = 0
    if nm != n_mels or stft.shape[0] != U or stft.shape[1] != n_fft // 2 + 1:
        raise ValueError("mel_db / stft shapes do not match")
    T_stft = stft.shape[2]
    T = min(T_pred, T_stft) if n_frames is None else n_frames
    if T != T_pred:
        # min() cut the prediction: use the [U, n_mels, T] layout of the concatenated, trimmed slices
        if spf:
            mel_db = mel_db.permute(0, 2, 1, 3).reshape(U, nm, T_pred)
        mel_db = mel_db[:, :, :T].contiguous()
        spf = 0
    out = torch.empty((U, hop_length * (T - 1)), dtype=torch.float32, device=mel_db.device)
    if U == 0:
        return out
    ctx = _lib.context(mel_db.device)
    with torch.cuda.device(mel_db.device):
        _lib.check(_lib.load().avse_istft(ctx.handle, _lib.ptr(mel_db), _lib.ptr(stft), U, int(T), int(T_stft), int(spf),
                                          int(sample_rate), int(n_fft), int(hop_length), int(n_mels), float(fmin),
                                          float(fmax), _lib.ptr(out), _lib.stream_handle(mel_db.device)), "avse_istft")
    return out


def act_exponent(model, layer):
    """The AVSE_F32_SPLIT activation exponent rule of csrc/capi.hip act_exponents for one layer: with M =
    max_c (|beta_c| + |gamma_c|) of its BatchNormalization, 0 for M in [2^-2, 2^8], else 3 - ceil-exponent(M) (M 2^e in
    (4, 8]), clamped to [-24, 24]."""
    g = np.abs(np.asarray(model.tensors[layer + "_bn/gamma"], np.float64))
    b = np.abs(np.asarray(model.tensors[layer + "_bn/beta"], np.float64))
    m = float(np.max(b + g))
    if not m > 0.0 or not np.isfinite(m) or 0.25 <= m <= 256.0:
        return 0
    return int(max(-24, min(24, 3 - np.frexp(m)[1])))


def _warn_concat_exponents(model):
    """a_conv5 and v_conv6 write the two halves of one concat row that enc_dense reads as one K, so they share one
    exponent, the smaller (capi.hip act_exponents).  When the halves' own rules disagree, the half that wanted the larger
    exponent is stored with fewer than the pairs' ~22 bits (its lo pieces run into the f16 subnormals): flag it at load
    time — the range guard reports overflow and NaN, not this precision loss."""
    ea, ev = act_exponent(model, "a_conv5"), act_exponent(model, "v_conv6")
    if ea != ev:
        import warnings
        warnings.warn(f"float32_split: the concat halves want activation exponents {ea} (a_conv5) and {ev} (v_conv6); "
                      f"both are stored at {min(ea, ev)}, so the {'audio' if ea > ev else 'video'} half's activations "
                      f"lose precision (BatchNormalization parameters outside [2^-2, 2^8]); use dtype float32 for exact "
                      "fp32 if that matters", RuntimeWarning, stacklevel=3)


class DeviceWeights:
    """avse_weights: BN-folded, GEMM-packed weights resident on one device."""

    def __init__(self, model, dtype="float32", device=None):
        if not isinstance(model, KerasModel):
            raise TypeError("model must be a KerasModel")
        self.dtype = DTYPES[dtype] if isinstance(dtype, str) else int(dtype)
        self.ctx = _lib.context(device)
        self.T, self.F = model.T, model.F
        self.last_range_bits = 0
        if self.dtype == _lib.AVSE_F32_SPLIT:
            _warn_concat_exponents(model)
        blob = model.to_blob()
        # the CDLL is held here: at interpreter exit the module globals may be gone before this object
        self._cdll = _lib.load()
        assert blob.size == blob_floats(self.T, self.F) == self._cdll.avse_weights_blob_floats_shape(self.T, self.F)
        self.handle = ctypes.c_void_p()
        with torch.cuda.device(self.ctx.device_index):
            _lib.check(_lib.load().avse_weights_load_shape(self.ctx.handle, blob.ctypes.data_as(ctypes.c_void_p),
                                                           blob.size, self.dtype, self.T, self.F,
                                                           ctypes.byref(self.handle)), "avse_weights_load_shape")

    @property
    def audio_shape(self):
        return (80, self.T)

    def act_exponents(self):
        """avse_weights_act_exponents: per plan layer, the power-of-two exponent its split-pair activations carry."""
        e = (ctypes.c_int * 20)()
        _lib.check(self._cdll.avse_weights_act_exponents(self.handle, e, 20), "avse_weights_act_exponents")
        return dict(zip(_lib.LAYER_NAMES, list(e)))

    def __del__(self):
        h, lib = getattr(self, "handle", None), getattr(self, "_cdll", None)
        if h is not None and h.value and lib is not None:
            lib.avse_weights_destroy(h)
            self.handle = None


def _check_forward_args(weights, audio, video, vnorm_mean, vnorm_std):
    _dev_f32(audio, "audio", (80, weights.T))
    N = audio.shape[0]
    if video is not None:
        _dev_f32(video, "video", (128, 128, weights.F))
        if video.shape[0] != N:
            raise ValueError("audio and video batch sizes differ")
    if (vnorm_mean is None) != (vnorm_std is None):
        raise ValueError("vnorm_mean and vnorm_std must both be given")
    if vnorm_mean is not None:
        if video is None:
            raise ValueError("video=None (all-zero video) takes no normaliser")
        _dev_f32(vnorm_mean, "vnorm_mean", (128, 128))
        _dev_f32(vnorm_std, "vnorm_std", (128, 128))
    devs = {weights.ctx.device_index, audio.device.index} | ({video.device.index} if video is not None else set())
    if len(devs) != 1:
        raise ValueError(f"weights live on cuda:{weights.ctx.device_index} but audio / video are on "
                         f"{audio.device} / {None if video is None else video.device}")
    return N


def forward(weights, audio, video, vnorm_mean=None, vnorm_std=None, out=None, checked=False, on_range="recompute"):
    """K2-K5: network forward.  audio [N, 80, 20], video [N, 128, 128, 5] float32 device tensors
    (video un-normalised when vnorm_* are given).  Returns [N, 80, 20] float32.  ([N, 80, T] / [N, 128, 128, F]
    for weights of another network shape, e.g. T = 24 at 29.97 fps.)

    video=None means an all-zero video input (BASELINE configs[2], the audio branch alone): the video
    encoder's output is then one constant vector, computed once per weights object and broadcast.

    checked=False (default): plain asynchronous avse_forward on torch's current stream, capturable in a graph; a
    float32_split forward leaves its range-guard bits in the context for Context.range_status / RangePipeline.
    checked=True: avse_forward_checked — BLOCKS the host until the stream has run the forward and, when an activation
    left the f16 pair range, recomputes the batch on the exact-fp32 kernels (on_range="recompute") or raises
    _lib.RangeError (on_range="error"); not allowed while the stream is capturing.  weights.last_range_bits holds the
    guard bits of the last checked call (0: every pair in range).  The synchronous reference-shaped API
    (network.SpeechEnhancementNetwork.predict / evaluate, the CLI predict) opts in for float32_split weights."""
    N = _check_forward_args(weights, audio, video, vnorm_mean, vnorm_std)
    if out is None:
        out = torch.empty((N, 80, weights.T), dtype=torch.float32, device=audio.device)
    _dev_f32(out, "out", (80, weights.T))
    if out.device != audio.device or out.shape[0] != N:
        raise ValueError(f"out must be [N, 80, {weights.T}] on the inputs' device")
    if N == 0:
        return out
    with torch.cuda.device(audio.device):
        if checked:
            mode = {"recompute": _lib.AVSE_RANGE_RECOMPUTE, "error": _lib.AVSE_RANGE_ERROR}[on_range]
            bits = ctypes.c_uint32()
            rc = _lib.load().avse_forward_checked(weights.ctx.handle, weights.handle, _lib.ptr(audio), _lib.ptr(video),
                                                  _lib.ptr(vnorm_mean), _lib.ptr(vnorm_std), N, _lib.ptr(out),
                                                  _lib.stream_handle(audio.device), mode, ctypes.byref(bits))
            weights.last_range_bits = bits.value
            _lib.check(rc, "avse_forward_checked")
            if bits.value:
                import warnings
                warnings.warn(f"float32_split forward of {N} clips: {_lib.range_bit_names(bits.value)} left the f16 pair "
                              "range; the batch was recomputed on the exact-fp32 kernels", RuntimeWarning, stacklevel=2)
        else:
            _lib.check(_lib.load().avse_forward(weights.ctx.handle, weights.handle, _lib.ptr(audio), _lib.ptr(video),
                                                _lib.ptr(vnorm_mean), _lib.ptr(vnorm_std), N, _lib.ptr(out),
                                                _lib.stream_handle(audio.device)), "avse_forward")
    return out


class RangePipeline:
    """Deferred range verification of unchecked float32_split forwards (avse_range_snapshot): after each forward,
    `submit(recompute)` enqueues a snapshot of the context's range guard into a pinned host word and an event; the
    snapshot of batch k is read once the stream has passed it — at the `depth`-th later submit, or at `drain()` — so the
    host never waits for the batch it just enqueued (avse_forward_checked waits for every batch before the next is
    launched).  A batch whose bits are set is recomputed by its `recompute` callable (e.g. ops.forward(...,
    checked=True) into the same output, which must then still hold that batch's inputs); `bits` accumulates every
    batch's guard bits and `recomputed` counts the batches redone."""

    def __init__(self, ctx, depth=2):
        self.ctx = ctx
        self.depth = max(1, int(depth))
        self.words = torch.zeros(self.depth, dtype=torch.int32, pin_memory=True)
        self.events = [torch.cuda.Event() for _ in range(self.depth)]
        self.pending = []
        self.k = 0
        self.bits = 0
        self.recomputed = 0

    def submit(self, recompute=None):
        slot = self.k % self.depth
        if len(self.pending) == self.depth:
            self._retire()
        dev = torch.device("cuda", self.ctx.device_index)
        with torch.cuda.device(dev):
            _lib.check(_lib.load().avse_range_snapshot(self.ctx.handle, _lib.stream_handle(dev),
                                                       ctypes.c_void_p(self.words.data_ptr() + 4 * slot)),
                       "avse_range_snapshot")
            self.events[slot].record()
        self.pending.append((slot, recompute))
        self.k += 1

    def _retire(self):
        slot, recompute = self.pending.pop(0)
        self.events[slot].synchronize()
        b = int(self.words[slot].item()) & 0xFFFFFFFF
        if b:
            self.bits |= b
            if recompute is not None:
                recompute()
                self.recomputed += 1

    def drain(self):
        while self.pending:
            self._retire()
        return self.bits


def forward_profile(weights, audio, video, vnorm_mean=None, vnorm_std=None, out=None):
    """forward() with HIP events between kernel launches (synchronises); returns (out, {stage: ms})."""
    N = _check_forward_args(weights, audio, video, vnorm_mean, vnorm_std)
    if out is None:
        out = torch.empty((N, 80, weights.T), dtype=torch.float32, device=audio.device)
    ms = (ctypes.c_float * _lib.AVSE_NUM_STAGES)()
    with torch.cuda.device(audio.device):
        _lib.check(_lib.load().avse_forward_profile(weights.ctx.handle, weights.handle, _lib.ptr(audio), _lib.ptr(video),
                                                    _lib.ptr(vnorm_mean), _lib.ptr(vnorm_std), N, _lib.ptr(out),
                                                    _lib.stream_handle(audio.device), ms), "avse_forward_profile")
    return out, dict(zip(_lib.STAGE_NAMES, [float(x) for x in ms]))


def video_normalize_(video, mean, std):
    """In place: video[s, :, :, f] = (video[s, :, :, f] - mean) / std (data_processor.py:208-212)."""
    _dev_f32(video, "video")
    _dev_f32(mean, "mean")
    _dev_f32(std, "std")
    S, H, W, F = video.shape
    if S == 0:
        return video
    ctx = _lib.context(video.device)
    with torch.cuda.device(video.device):
        _lib.check(_lib.load().avse_video_normalize(ctx.handle, _lib.ptr(video), S, H, W, F, _lib.ptr(mean),
                                                    _lib.ptr(std), _lib.stream_handle(video.device)),
                   "avse_video_normalize")
    return video


def mse(pred, target):
    """Keras mean_squared_error over every element -> 0-dim device tensor."""
    _dev_f32(pred, "pred")
    _dev_f32(target, "target")
    if pred.numel() != target.numel():
        raise ValueError("pred/target sizes differ")
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    ctx = _lib.context(pred.device)
    with torch.cuda.device(pred.device):
        _lib.check(_lib.load().avse_mse(ctx.handle, _lib.ptr(pred), _lib.ptr(target), pred.numel(), _lib.ptr(loss),
                                        _lib.stream_handle(pred.device)), "avse_mse")
    return loss


def to_device(x, device=None):
    """numpy / tensor -> contiguous float32 device tensor (host->device copy only)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.float32).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev)


class Trainer:
    """libavse training step (avse_trainer_*, train.hip): one Keras fit step of SpeechEnhancementNetwork.train
    (network.py:177-206) — BatchNormalization on batch statistics, Dropout after each video pooling, MSE, Adam.
    Parameters / gradients / Adam moments stay on the device in the canonical blob layout."""

    def __init__(self, model, max_batch=16, device=None):
        if not isinstance(model, KerasModel):
            raise TypeError("model must be a KerasModel")
        self.ctx = _lib.context(device)
        self.max_batch = int(max_batch)
        self.T, self.F = model.T, model.F
        blob = model.to_blob()
        self._cdll = _lib.load()   # held for __del__ (see DeviceWeights)
        self.handle = ctypes.c_void_p()
        with torch.cuda.device(self.ctx.device_index):
            _lib.check(_lib.load().avse_trainer_create_shape(self.ctx.handle, blob.ctypes.data_as(ctypes.c_void_p),
                                                             blob.size, self.max_batch, self.T, self.F,
                                                             ctypes.byref(self.handle)), "avse_trainer_create_shape")
        self._loss = torch.zeros((), dtype=torch.float32, device=torch.device("cuda", self.ctx.device_index))

    def step(self, audio, video, target, vnorm_mean=None, vnorm_std=None, lr=5e-4, dropout=0.25, seed=0,
             grads_only=False):
        """One fit step on a batch: audio / target [N, 80, 20], video [N, 128, 128, 5] (raw crops when vnorm_* are
        given) float32 device tensors.  Returns the batch MSE before the update as a 0-dim device tensor."""
        _dev_f32(audio, "audio", (80, self.T))
        _dev_f32(target, "target", (80, self.T))
        _dev_f32(video, "video", (128, 128, self.F))
        N = audio.shape[0]
        if video.shape[0] != N or target.shape[0] != N:
            raise ValueError("audio, video and target batch sizes differ")
        if N > self.max_batch:
            raise ValueError(f"batch of {N} exceeds the trainer's max_batch {self.max_batch}")
        if (vnorm_mean is None) != (vnorm_std is None):
            raise ValueError("vnorm_mean and vnorm_std must both be given")
        devs = {self.ctx.device_index, audio.device.index, video.device.index, target.device.index}
        if len(devs) != 1:
            raise ValueError("trainer and batch tensors must share one device")
        with torch.cuda.device(audio.device):
            _lib.check(_lib.load().avse_trainer_step(
                self.handle, _lib.ptr(audio), _lib.ptr(video), _lib.ptr(target), _lib.ptr(vnorm_mean),
                _lib.ptr(vnorm_std), N, float(lr), float(dropout), int(seed) & 0xFFFFFFFF,
                _lib.AVSE_TRAIN_GRADS_ONLY if grads_only else 0, _lib.ptr(self._loss),
                _lib.stream_handle(audio.device)), "avse_trainer_step")
        return self._loss.clone()

    def _read(self, what):
        out = np.empty(blob_floats(self.T, self.F), dtype=np.float32)
        _lib.check(_lib.load().avse_trainer_read(self.handle, what, out.ctypes.data_as(ctypes.c_void_p), out.size),
                   "avse_trainer_read")
        return out

    def model(self):
        """Current parameters (incl. BN moving statistics) as a KerasModel."""
        return KerasModel.from_blob(self._read(_lib.AVSE_TRAIN_PARAMS), self.T, self.F)

    def gradients(self):
        """Gradients of the last step, {tensor name: array} (moving statistics: zero)."""
        return KerasModel.from_blob(self._read(_lib.AVSE_TRAIN_GRADS), self.T, self.F).tensors

    @property
    def iterations(self):
        v = ctypes.c_int64()
        _lib.check(_lib.load().avse_trainer_iterations(self.handle, ctypes.byref(v)), "avse_trainer_iterations")
        return v.value

    def __del__(self):
        h, lib = getattr(self, "handle", None), getattr(self, "_cdll", None)
        if h is not None and h.value and lib is not None:
            lib.avse_trainer_destroy(h)
            self.handle = None
