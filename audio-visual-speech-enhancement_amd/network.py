"""SpeechEnhancementNetwork — drop-in for /root/reference/network.py's inference API on MI355X.

build / predict / evaluate / load / save keep the reference's signatures and tensor shapes
(`predict` takes [N, 80, 20] + [N, 128, 128, 5] and returns np.squeeze of [N, 80, 20, 1]; a network built for
another frame rate — build((80, 24), (128, 128, 5 or 6)) at 29.97 / 30 fps — takes and returns its own shapes).
The forward pass is libavse's avse_forward (HIP kernels); there is no Keras and no CPU fallback.
train (network.py:177-206) runs Keras-semantics fit steps on libavse's training step (fit.py, csrc/train.hip).
"""
import numpy as np
import torch

from . import _lib, ops
from .model import KerasModel, shape_supported


class SpeechEnhancementNetwork(object):

    def __init__(self, model, compute_dtype="float32", device=None):
        self.__model = model
        self.__compute_dtype = compute_dtype
        self.__device = device
        self.__dw = None

    @property
    def model(self):
        return self.__model

    def device_weights(self):
        if self.__dw is None:
            self.__dw = ops.DeviceWeights(self.__model, self.__compute_dtype, self.__device)
        return self.__dw

    @classmethod
    def build(cls, audio_spectrogram_shape, video_shape, seed=0, compute_dtype="float32"):
        """network.py:17-40 — fresh Keras-default-initialised network for these input shapes: audio [80, T] (T = 20 at
        25 fps, 24 at 29.97 / 30 fps), video [128, 128, F] (F = 5, or 6 at 30 fps).  The layer widths follow the
        shapes as in Keras (model.layers).  Shapes whose decoder cannot reproduce 80 x T (T not a multiple of 4)
        raise NotImplementedError."""
        a, v = tuple(int(x) for x in audio_spectrogram_shape), tuple(int(x) for x in video_shape)
        if len(a) != 2 or a[0] != 80 or len(v) != 3 or v[:2] != (128, 128) or not shape_supported(a[1], v[2]):
            raise NotImplementedError(
                f"audio [80, T] with T a multiple of 4 and video [128, 128, F <= 8] are implemented (16 kHz, 200-ms "
                f"slices: T = 20 at 25 fps, 24 at 29.97 / 30 fps); got {a}, {v}")
        return SpeechEnhancementNetwork(KerasModel.init(seed=seed, audio_shape=a, video_shape=v), compute_dtype)

    def train(self, train_mixed_spectrograms, train_video_samples, train_speech_spectrograms,
              validation_mixed_spectrograms, validation_video_samples, validation_speech_spectrograms,
              model_cache_path, tensorboard_dir=None, batch_size=16, epochs=1000, lr=5e-4, seed=0, verbose=1):
        """network.py:177-206: Model.fit(batch_size=16, epochs=1000) with ModelCheckpoint(model_cache_path),
        ReduceLROnPlateau(val_loss, 0.5, patience 5), EarlyStopping(val_loss, min_delta 0.01, patience 10) on the
        Adam(5e-4) / MSE compilation of network.py:35-36.  Video samples are expected normalised (as the
        reference's speech_enhancer.train does in place).  tensorboard_dir is accepted and unused (no
        TensorFlow).  The trained parameters replace this network's; returns the per-epoch history."""
        from .fit import fit
        model, history = fit(self.__model, (train_mixed_spectrograms, train_video_samples, train_speech_spectrograms),
                             (validation_mixed_spectrograms, validation_video_samples, validation_speech_spectrograms),
                             model_cache_path=model_cache_path, batch_size=batch_size, epochs=epochs, lr=lr, seed=seed,
                             device=self.__device, verbose=verbose)
        self.__model = model
        self.__dw = None
        return history

    def predict_device(self, mixed_spectrograms, video_samples, video_normalizer=None, checked=None):
        """Device-tensor forward: [N, 80, T] x [N, 128, 128, F] -> [N, 80, T] (no squeeze).  checked (default: on for
        float32_split weights, whose range guard is then read before returning) as in ops.forward."""
        a = ops.to_device(mixed_spectrograms, self.__device)
        v = None if video_samples is None else ops.to_device(video_samples, a.device)   # None: all-zero video
        m = s = None
        if video_normalizer is not None:
            m, s = video_normalizer.device_stats(a.device)
        dw = self.device_weights()
        if checked is None:
            checked = dw.dtype == _lib.AVSE_F32_SPLIT
        return ops.forward(dw, a, v, m, s, checked=checked)

    def predict(self, mixed_spectrograms, video_samples, video_normalizer=None):
        """network.py:208-212.  video_normalizer (optional) fuses VideoNormalizer.normalize into the
        first video conv instead of normalising the array in place beforehand."""
        out = self.predict_device(mixed_spectrograms, video_samples, video_normalizer)
        if isinstance(mixed_spectrograms, torch.Tensor):
            return out.squeeze()
        return np.squeeze(out.cpu().numpy())

    def evaluate(self, mixed_spectrograms, video_samples, speech_spectrograms, video_normalizer=None):
        """network.py:214-220: mean squared error of the prediction over every element."""
        pred = self.predict_device(mixed_spectrograms, video_samples, video_normalizer)
        target = ops.to_device(speech_spectrograms, pred.device).reshape(pred.shape)
        return float(ops.mse(pred, target).item())

    def predict_and_evaluate(self, mixed_spectrograms, video_samples, speech_spectrograms, video_normalizer=None):
        """predict() and evaluate() from ONE forward: (squeezed prediction, MSE of that prediction).
        speech_enhancer.py:76-79 runs the two on the same input; the loss is the same value."""
        pred = self.predict_device(mixed_spectrograms, video_samples, video_normalizer)
        target = ops.to_device(speech_spectrograms, pred.device).reshape(pred.shape)
        loss = float(ops.mse(pred, target).item())
        if isinstance(mixed_spectrograms, torch.Tensor):
            return pred.squeeze(), loss
        return np.squeeze(pred.cpu().numpy()), loss

    @staticmethod
    def load(model_cache_path, compute_dtype="float32"):
        """network.py:222-226 (own safetensors format; Keras HDF5 needs the converter)."""
        return SpeechEnhancementNetwork(KerasModel.load(model_cache_path), compute_dtype)

    def save(self, model_cache_path):
        """network.py:228-229."""
        self.__model.save(model_cache_path)
