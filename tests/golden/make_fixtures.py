"""Generate golden fixtures by executing the REFERENCE's own Python code (this container only).

/root/reference/data_processor.py and network.py import librosa / keras / mediaio / facedetection,
none of which exist here (ordinary ModuleNotFoundError, not a permission denial).  We inject
*recording stubs* for those modules and run the reference's own functions, capturing what its code
decides by itself:

  slicing.json       preprocess_audio_signal (data_processor.py:35-57): padded/truncated length,
                     the (n_fft, hop) it passes to librosa.core.stft, and which STFT frame ids land
                     in which slice (the stub STFT encodes frame id t as the value t), for several
                     lengths and frame rates; reconstruct_speech_signal (:60-74): the shapes and hop
                     it hands to pinv / istft.
  network_spec.json  SpeechEnhancementNetwork.build((80, 20), (128, 128, 5)) (network.py:17-40)
                     against a symbolic Keras stub: every layer constructor call in order with its
                     arguments and the propagated output shape, plus the compile() call.
  network_spec_2997fps.json / network_spec_30fps.json
                     the same for the shapes the reference's preprocessing produces at 29.97 fps
                     ((80, 24), (128, 128, 5)) and 30 fps ((80, 24), (128, 128, 6)) (data_processor.py:24, :44-52).

The reference never travels: only these JSON outputs (data) are committed.
Run:  python tests/golden/make_fixtures.py
"""
import json
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _clear(names):
    for n in list(sys.modules):
        if n in names or any(n.startswith(p + ".") for p in names):
            del sys.modules[n]


# ------------------------------------------------------------------------------------------
# data_processor.py with stub librosa / mediaio / facedetection
# ------------------------------------------------------------------------------------------
def slicing_fixture():
    calls = []
    librosa = types.ModuleType("librosa")
    core = types.ModuleType("librosa.core")
    filters = types.ModuleType("librosa.filters")

    def stft(y, n_fft, hop_length):
        T = 1 + (len(y) + 2 * (n_fft // 2) - n_fft) // hop_length
        calls.append({"fn": "stft", "len": int(len(y)), "n_fft": int(n_fft), "hop_length": int(hop_length), "T": T})
        return np.tile(np.arange(T, dtype=np.complex64), (1 + n_fft // 2, 1))   # value = frame id

    def mel(sr, n_fft, n_mels, fmin, fmax):
        calls.append({"fn": "mel", "sr": sr, "n_fft": int(n_fft), "n_mels": n_mels, "fmin": fmin, "fmax": fmax})
        return np.eye(n_mels, 1 + n_fft // 2)                                    # row m <- bin m

    def istft(S, hop_length):
        calls.append({"fn": "istft", "shape": list(S.shape), "hop_length": int(hop_length)})
        n_fft = 2 * (S.shape[0] - 1)
        return np.zeros(hop_length * (S.shape[1] - 1) + n_fft - 2 * (n_fft // 2))

    core.stft = stft
    core.magphase = lambda D: (np.abs(D), np.ones_like(D))
    filters.mel = mel
    librosa.core = core
    librosa.filters = filters
    librosa.amplitude_to_db = lambda S: S
    librosa.db_to_amplitude = lambda S: S
    librosa.istft = istft

    class AudioSignal:
        def __init__(self, data, sample_rate):
            self.data = np.asarray(data, dtype=np.float64)
            self.sr = sample_rate

        def get_sample_rate(self):
            return self.sr

        def get_number_of_samples(self):
            return len(self.data)

        def pad_with_zeros(self, n):
            self.data = np.concatenate([self.data, np.zeros(n - len(self.data))])

        def truncate(self, n):
            self.data = self.data[:n]

        def get_data(self, channel_index=None):
            return self.data

    mods = {"librosa": librosa, "librosa.core": core, "librosa.filters": filters,
            "facedetection": types.ModuleType("facedetection"),
            "facedetection.face_detection": types.ModuleType("facedetection.face_detection"),
            "mediaio": types.ModuleType("mediaio"), "mediaio.audio_io": types.ModuleType("mediaio.audio_io"),
            "mediaio.video_io": types.ModuleType("mediaio.video_io"),
            "multiprocess": types.ModuleType("multiprocess")}
    mods["facedetection.face_detection"].FaceDetector = object
    mods["mediaio.audio_io"].AudioSignal = AudioSignal
    mods["mediaio.audio_io"].AudioMixer = object
    mods["mediaio.video_io"].VideoFileReader = object
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    try:
        _clear(["data_processor"])
        import data_processor as dp
        cases = []
        for (L, n_slices, fps) in [(48000, 15, 25.0), (47000, 15, 25.0), (50000, 15, 25.0), (3200, 1, 25.0),
                                   (3199, 1, 25.0), (16000, 5, 25.0), (32000, 10, 29.97), (31000, 10, 29.97),
                                   (64000, 20, 30.0), (8000, 2, 24.0)]:
            sig = AudioSignal(np.zeros(L), 16000)
            del calls[:]
            out = dp.preprocess_audio_signal(sig, 200, n_slices, fps)
            st = [c for c in calls if c["fn"] == "stft"][0]
            frame_ids = np.real(out[:, 0, :]).astype(int)        # [n_slices, spf] frame ids
            cases.append({"n_samples_in": L, "n_video_slices": n_slices, "fps": fps,
                          "signal_length": sig.get_number_of_samples(), "n_fft": st["n_fft"],
                          "hop_length": st["hop_length"], "n_frames": st["T"], "out_shape": list(out.shape),
                          "frame_ids": frame_ids.tolist()})
        recon = []
        for (n_slices, fps) in [(15, 25.0), (10, 29.97)]:
            del calls[:]
            g = cases[0] if fps == 25.0 else cases[6]
            mixed = AudioSignal(np.zeros(g["signal_length"]), 16000)
            dp.reconstruct_speech_signal(mixed, np.zeros((n_slices, 80, g["out_shape"][2])), fps)
            recon.append({"n_slices": n_slices, "fps": fps, "calls": [c for c in calls if c["fn"] != "mel"]})
        return {"source": "data_processor.py:35-74 executed with stub librosa/mediaio (tests/golden/make_fixtures.py)",
                "preprocess_audio_signal": cases, "reconstruct_speech_signal": recon}
    finally:
        sys.path.remove(REF)
        _clear(["data_processor"])
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


# ------------------------------------------------------------------------------------------
# network.py with a symbolic keras stub
# ------------------------------------------------------------------------------------------
def network_fixture(audio_shape=(80, 20), video_shape=(128, 128, 5)):
    log = []

    class Shape(tuple):
        def as_list(self):
            return list(self)

        def __getitem__(self, i):
            r = tuple.__getitem__(self, i)
            return Shape(r) if isinstance(i, slice) else r

    class Sym:
        def __init__(self, shape):
            self.shape = Shape((None,) + tuple(shape))
            self._keras_shape = self.shape

    def layer(kind, shape_fn):
        class L:
            def __init__(self, *a, **k):
                self.a, self.k = a, k

            def __call__(self, x):
                ins = [t.shape[1:] for t in (x if isinstance(x, list) else [x])]
                out = shape_fn(self, *ins)
                log.append({"layer": kind, "args": [list(v) if isinstance(v, tuple) else v for v in self.a],
                            "kwargs": {k: (list(v) if isinstance(v, tuple) else v) for k, v in self.k.items()},
                            "in": [list(s) for s in ins], "out": list(out)})
                return Sym(out)
        return L

    def conv(self, x):
        s = self.k.get("strides", (1, 1))
        return (math.ceil(x[0] / s[0]), math.ceil(x[1] / s[1]), self.a[0])

    def deconv(self, x):
        s = self.k.get("strides", (1, 1))
        return (x[0] * s[0], x[1] * s[1], self.a[0])

    def pool(self, x):
        s = self.k["strides"]
        return (math.ceil(x[0] / s[0]), math.ceil(x[1] / s[1]), x[2])

    keras = types.ModuleType("keras")
    layers = types.ModuleType("keras.layers")
    merge = types.ModuleType("keras.layers.merge")
    models = types.ModuleType("keras.models")
    callbacks = types.ModuleType("keras.callbacks")
    optimizers = types.ModuleType("keras.optimizers")

    def Input(shape):
        log.append({"layer": "Input", "out": list(shape)})
        return Sym(tuple(shape))

    layers.Input = Input
    layers.Dense = layer("Dense", lambda s, x: (s.a[0],))
    layers.Convolution2D = layer("Conv2D", conv)
    layers.Deconvolution2D = layer("Conv2DTranspose", deconv)
    layers.MaxPooling2D = layer("MaxPooling2D", pool)
    layers.Dropout = layer("Dropout", lambda s, x: x)
    layers.Flatten = layer("Flatten", lambda s, x: (int(np.prod(x)),))
    layers.BatchNormalization = layer("BatchNormalization", lambda s, x: x)
    layers.LeakyReLU = layer("LeakyReLU", lambda s, x: x)
    layers.Reshape = layer("Reshape", lambda s, x: tuple(s.a[0]))

    def concatenate(xs):
        out = (sum(t.shape[1] for t in xs),)
        log.append({"layer": "Concatenate", "in": [list(t.shape[1:]) for t in xs], "out": list(out)})
        return Sym(out)

    merge.concatenate = concatenate

    class Model:
        def __init__(self, inputs, outputs):
            self.o = outputs
            log.append({"layer": "Model", "out": list(outputs.shape[1:])})

        def summary(self):
            pass

        def compile(self, **k):
            log.append({"layer": "compile", "loss": k.get("loss"), "optimizer": list(k.get("optimizer"))})

        def __call__(self, x):
            return Sym(self.o.shape[1:])

    models.Model = Model
    models.load_model = None
    for n in ["EarlyStopping", "ReduceLROnPlateau", "ModelCheckpoint", "TensorBoard"]:
        setattr(callbacks, n, object)
    optimizers.adam = lambda lr: ("adam", lr)
    keras.optimizers = optimizers
    mods = {"keras": keras, "keras.layers": layers, "keras.layers.merge": merge, "keras.models": models,
            "keras.callbacks": callbacks, "keras.optimizers": optimizers}
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    sys.path.insert(0, REF)
    try:
        _clear(["network"])
        import network
        network.SpeechEnhancementNetwork.build(audio_shape, video_shape)
        return {"source": "network.py:17-175 executed against a symbolic keras stub (tests/golden/make_fixtures.py)",
                "build_args": [list(audio_shape), list(video_shape)], "graph": log}
    finally:
        sys.path.remove(REF)
        _clear(["network"])
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def main():
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not present: fixtures can only be regenerated in the build container")
    with open(os.path.join(HERE, "slicing.json"), "w") as f:
        json.dump(slicing_fixture(), f, indent=1)
    for name, a, v in [("network_spec.json", (80, 20), (128, 128, 5)),
                       ("network_spec_2997fps.json", (80, 24), (128, 128, 5)),
                       ("network_spec_30fps.json", (80, 24), (128, 128, 6))]:
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(network_fixture(a, v), f, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))
    print("wrote slicing.json, network_spec*.json")


if __name__ == "__main__":
    main()
