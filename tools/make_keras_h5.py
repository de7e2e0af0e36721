"""Test helper: write avse canonical tensors (an .npz, allow_pickle=False) as a Keras-2-layout HDF5 model file,
the layout `Model.save` of network.py:228-229 produces — root attrs `keras_version` / `backend` /
`model_config`, `model_weights` with `layer_names` = [input_1, input_2, model_1, model_2], the encoder's and
decoder's weights nested in their sub-model groups as `<layer>/<param>:0` datasets listed in `weight_names`.
Auto-names start at `--offset` (a Keras session that built other layers first numbers from there).

    /opt/conda/bin/python3.9 tools/make_keras_h5.py weights.npz model.h5py [--offset N]

No trained reference model ships with the reference, so tests/test_keras_h5.py round-trips through this
writer: the converter's mapping is pinned to the reference's layer creation order, not to a real file.
"""
import argparse
import json

import h5py
import numpy as np

from keras_h5_to_avse import KERAS_PREFIX, _model_module

ENCODER = ("a_conv", "v_conv", "enc_dense")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--offset", type=int, default=1)
    ap.add_argument("--corrupt", default="", help="tensor name whose kernel gets a wrong shape (negative test)")
    a = ap.parse_args()
    M = _model_module()
    t = np.load(a.src, allow_pickle=False)
    counters = {}

    def name(prefix):
        counters[prefix] = counters.get(prefix, a.offset - 1) + 1
        return f"{prefix}_{counters[prefix]}"

    groups = {"model_1": [], "model_2": []}       # (keras layer name, [(param, array)])
    config = {"model_1": [], "model_2": []}
    for L in M.LAYERS:                            # creation order of network.py:17-175
        sub = "model_1" if L.name.startswith(ENCODER) else "model_2"
        kname = name(KERAS_PREFIX[L.kind])
        k = t[L.name + "/kernel"]
        if a.corrupt == L.name:
            k = k[..., :-1]
        groups[sub].append((kname, [("kernel", k), ("bias", t[L.name + "/bias"])]))
        config[sub].append({"class_name": {"conv": "Conv2D", "deconv": "Conv2DTranspose", "dense": "Dense"}[L.kind],
                            "name": kname})
        if L.bn_channels:
            bname = name("batch_normalization")
            groups[sub].append((bname, [(q, t[f"{L.name}_bn/{q}"]) for q in ("gamma", "beta", "moving_mean",
                                                                             "moving_variance")]))
            config[sub].append({"class_name": "BatchNormalization", "name": bname})
    with h5py.File(a.dst, "w") as f:
        f.attrs["keras_version"] = b"2.0.8"
        f.attrs["backend"] = b"tensorflow"
        f.attrs["model_config"] = json.dumps({"class_name": "Model", "config": {"layers": [
            {"class_name": "InputLayer", "name": "input_1"}, {"class_name": "InputLayer", "name": "input_2"},
            {"class_name": "Model", "name": "model_1", "config": {"layers": config["model_1"]}},
            {"class_name": "Model", "name": "model_2", "config": {"layers": config["model_2"]}}]}}).encode()
        mw = f.create_group("model_weights")
        mw.attrs["layer_names"] = np.array([b"input_1", b"input_2", b"model_1", b"model_2"])
        mw.attrs["backend"] = b"tensorflow"
        mw.attrs["keras_version"] = b"2.0.8"
        for n in ("input_1", "input_2"):
            mw.create_group(n).attrs["weight_names"] = np.array([], dtype="S1")
        for sub, layers in groups.items():
            g = mw.create_group(sub)
            names = [f"{kn}/{p}:0" for kn, ps in layers for p, _ in ps]
            g.attrs["weight_names"] = np.array([n.encode() for n in names])
            for kn, ps in layers:
                for p, arr in ps:
                    g.create_dataset(f"{kn}/{p}:0", data=np.asarray(arr, np.float32))
        # an optimizer state group the converter must ignore
        f.create_group("optimizer_weights").create_dataset("training/Adam/conv2d_1/kernel/m:0", data=np.zeros(3))


if __name__ == "__main__":
    main()
