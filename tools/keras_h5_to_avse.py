"""Convert a Keras HDF5 model of the reference network (network.py:222-229 `model.save` / `load_model`,
cache/models/<model>/model.h5py, speech_enhancer.py:120-122) into this build's weight file
(safetensors, the canonical tensor names of avse_amd/model.py).

    /opt/conda/bin/python3.9 tools/keras_h5_to_avse.py model.h5py model.avse.safetensors

Needs h5py (in this image only under /opt/conda/bin/python3.9; HDF5 is plain data — nothing in the file is
executed).  Offline step, like SURVEY.md §8(f) 2 asks: the product loads the safetensors output.

Mapping.  Keras 2 names auto-created layers `<class prefix>_<n>` in creation order (conv2d, conv2d_transpose,
dense, batch_normalization); a full-model file stores them under `model_weights/`, the encoder's and decoder's
weights nested in their sub-model groups (`model_weights/model_1/conv2d_1/kernel:0`).  The creation order of
network.py:17-175 — the order of avse_amd/model.py's LAYERS, checked against the stub-executed layer graph in
tests/golden/network_spec.json — assigns each class's layers by their index, whatever the session's counter
offset was.  Every tensor's shape is checked against the layer table.  Weights-only files
(`save_weights`: layer groups at the root) are read the same way.
"""
import argparse
import importlib.util
import json
import os
import re
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model_module():
    # model.py imports only json / collections / numpy: load it by path (no torch in this interpreter)
    path = os.path.join(ROOT, "audio-visual-speech-enhancement_amd", "model.py")
    spec = importlib.util.spec_from_file_location("avse_model_table", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


KERAS_PREFIX = {"conv": "conv2d", "deconv": "conv2d_transpose", "dense": "dense"}
PARAMS = {"kernel": "kernel", "bias": "bias", "gamma": "gamma", "beta": "beta", "moving_mean": "moving_mean",
          "moving_variance": "moving_variance"}
NAME_RE = re.compile(r"^(conv2d_transpose|conv2d|dense|batch_normalization)_(\d+)$")


def collect_layers(h5):
    """{keras layer name: {param: ndarray}} from a Keras 2 HDF5 file (full model or weights only)."""
    import h5py
    root = h5["model_weights"] if "model_weights" in h5 else h5
    layers = {}

    def visit(name, obj):
        if not isinstance(obj, h5py.Dataset):
            return
        parts = name.split("/")
        if len(parts) < 2 or "optimizer_weights" in parts:
            return
        layer, param = parts[-2], parts[-1].split(":")[0]
        if NAME_RE.match(layer) and param in PARAMS:
            layers.setdefault(layer, {})[param] = np.asarray(obj[()], dtype=np.float32)

    root.visititems(visit)
    return layers


def map_layers(layers, M):
    """Keras layer dict -> OrderedDict of avse canonical tensors (raises on any mismatch)."""
    by_prefix = {}
    for name in layers:
        prefix, idx = NAME_RE.match(name).groups()
        by_prefix.setdefault(prefix, []).append((int(idx), name))
    for v in by_prefix.values():
        v.sort()
    want = {p: [L for L in M.LAYERS if KERAS_PREFIX[L.kind] == p] for p in ("conv2d", "conv2d_transpose", "dense")}
    want_bn = [L for L in M.LAYERS if L.bn_channels]
    out = {}
    for prefix, ours in list(want.items()) + [("batch_normalization", want_bn)]:
        got = by_prefix.get(prefix, [])
        if len(got) != len(ours):
            raise ValueError(f"{prefix}: the file has {len(got)} layers, the reference network has {len(ours)}")
        for (_, kname), L in zip(got, ours):
            p = layers[kname]
            if prefix == "batch_normalization":
                for q in ("gamma", "beta", "moving_mean", "moving_variance"):
                    a = p.get(q)
                    if a is None or a.shape != (L.bn_channels,):
                        raise ValueError(f"{kname}/{q}: expected ({L.bn_channels},) for {L.name}_bn")
                    out[f"{L.name}_bn/{q}"] = a
            else:
                ks = M.kernel_shape(L)
                if p.get("kernel") is None or p["kernel"].shape != ks:
                    raise ValueError(f"{kname}/kernel: expected {ks} for {L.name}, got "
                                     f"{None if p.get('kernel') is None else p['kernel'].shape}")
                if p.get("bias") is None or p["bias"].shape != (L.cout,):
                    raise ValueError(f"{kname}/bias: expected ({L.cout},) for {L.name}")
                out[f"{L.name}/kernel"] = p["kernel"]
                out[f"{L.name}/bias"] = p["bias"]
    missing = [n for n, _ in M.tensor_names() if n not in out]
    if missing:
        raise ValueError(f"missing tensors: {missing}")
    return [(n, out[n]) for n, _ in M.tensor_names()]


def write_safetensors(path, tensors, metadata):
    """safetensors layout: u64 header length, JSON header, raw little-endian data (F32)."""
    header, off = {"__metadata__": metadata}, 0
    blobs = []
    for name, a in tensors:
        b = np.ascontiguousarray(a, dtype="<f4").tobytes()
        header[name] = {"dtype": "F32", "shape": list(a.shape), "data_offsets": [off, off + len(b)]}
        off += len(b)
        blobs.append(b)
    h = json.dumps(header, separators=(",", ":")).encode()
    h += b" " * ((8 - len(h) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(h)))
        f.write(h)
        for b in blobs:
            f.write(b)


def convert(src, dst):
    import h5py
    M = _model_module()
    with h5py.File(src, "r") as h5:
        tensors = map_layers(collect_layers(h5), M)
    write_safetensors(dst, tensors, {"format": M.FORMAT, "layers": json.dumps([L.name for L in M.LAYERS]),
                                     "source": os.path.basename(src)})
    return len(tensors)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("src", help="Keras HDF5 model (model.h5py)")
    ap.add_argument("dst", help="output safetensors")
    a = ap.parse_args(argv)
    n = convert(a.src, a.dst)
    print(f"wrote {n} tensors to {a.dst}")


if __name__ == "__main__":
    sys.exit(main())
