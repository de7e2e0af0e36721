"""Keras HDF5 weight import (network.py:222-229): tools/keras_h5_to_avse.py maps a
Keras-2-layout model file onto the canonical tensors, by each Keras class's creation order
(network.py:17-175, as recorded in tests/golden/network_spec.json).

h5py exists in this image only under /opt/conda/bin/python3.9, so the converter (an offline step) and the
fixture writer run there; the tests skip elsewhere.  No trained reference model ships with the reference:
the files are written by tools/make_keras_h5.py in the layout Keras 2's Model.save produces — the mapping
is pinned to the reference's layer order, the file layout to Keras 2's published format (parity unpinned
against a real Keras-written file)."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY39 = "/opt/conda/bin/python3.9"


def _h5_python():
    if not os.path.exists(PY39):
        return None
    r = subprocess.run([PY39, "-c", "import h5py"], capture_output=True)
    return PY39 if r.returncode == 0 else None


H5PY = _h5_python()
needs_h5py = pytest.mark.skipif(H5PY is None, reason="no interpreter with h5py (converter is an offline step)")


def _run(*args):
    return subprocess.run([H5PY, *args], capture_output=True, text=True, cwd=os.path.join(ROOT, "tools"))


def _write_npz(model, path):
    np.savez(path, **{k: v for k, v in model.tensors.items()})


def test_layer_order_matches_reference_graph():
    """model.py's LAYERS (the converter's assignment order) = the weight layers of the stub-executed
    reference graph, class by class."""
    from avse_amd.model import LAYERS
    graph = json.load(open(os.path.join(ROOT, "tests", "golden", "network_spec.json")))["graph"]
    kinds = {"Conv2D": "conv", "Conv2DTranspose": "deconv", "Dense": "dense"}
    ref = [kinds[g["layer"]] for g in graph if g["layer"] in kinds]
    assert ref == [L.kind for L in LAYERS]
    n_bn = sum(1 for g in graph if g["layer"] == "BatchNormalization")
    assert n_bn == sum(1 for L in LAYERS if L.bn_channels)
    # each BN follows its weight layer in the graph
    seq = [g["layer"] for g in graph if g["layer"] in kinds or g["layer"] == "BatchNormalization"]
    owners = []
    for i, s in enumerate(seq):
        if s == "BatchNormalization":
            owners.append(sum(1 for x in seq[:i] if x in kinds) - 1)
    assert owners == [i for i, L in enumerate(LAYERS) if L.bn_channels]


@needs_h5py
@pytest.mark.parametrize("offset", [1, 7])
def test_keras_h5_round_trip(tmp_path, offset):
    from avse_amd.model import KerasModel
    m = KerasModel.init(seed=offset, randomize=True)
    npz, h5, st = tmp_path / "w.npz", tmp_path / "model.h5py", tmp_path / "model.safetensors"
    _write_npz(m, npz)
    r = _run("make_keras_h5.py", str(npz), str(h5), "--offset", str(offset))
    assert r.returncode == 0, r.stderr
    r = _run("keras_h5_to_avse.py", str(h5), str(st))
    assert r.returncode == 0, r.stderr
    got = KerasModel.load(str(st))
    for k, v in m.tensors.items():
        assert np.array_equal(got.tensors[k], v), k
    # the product refuses the HDF5 file itself and names the converter
    with pytest.raises(ValueError, match="keras_h5_to_avse"):
        KerasModel.load(str(h5))


@needs_h5py
def test_keras_h5_shape_mismatch_is_an_error(tmp_path):
    from avse_amd.model import KerasModel
    m = KerasModel.init(seed=2)
    npz, h5, st = tmp_path / "w.npz", tmp_path / "model.h5py", tmp_path / "model.safetensors"
    _write_npz(m, npz)
    assert _run("make_keras_h5.py", str(npz), str(h5), "--corrupt", "v_conv3").returncode == 0
    r = _run("keras_h5_to_avse.py", str(h5), str(st))
    assert r.returncode != 0 and "v_conv3" in r.stderr
    assert not st.exists()


@needs_h5py
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float32_split"])
def test_converted_keras_h5_runs_forward_against_oracle(tmp_path, gpu, dtype):
    """SpeechEnhancementNetwork.load of a Keras model file (network.py:222-226), end to end: a Keras-2-layout
    HDF5 file -> tools/keras_h5_to_avse.py -> KerasModel.load -> libavse forward (exact fp32 and the credited
    float32_split dtype, the output layer at dB scale), against the float64 oracle run on the ORIGINAL tensors (so a
    mis-mapped layer shows up as a forward error, not only as a tensor mismatch)."""
    import torch
    from avse_amd import ops
    from avse_amd.model import KerasModel
    from oracle import keras_ref as K
    from test_gpu_forward import db_scale
    m = db_scale(KerasModel.init(seed=5, randomize=True))
    npz, h5, st = tmp_path / "w.npz", tmp_path / "model.h5py", tmp_path / "model.safetensors"
    _write_npz(m, npz)
    assert _run("make_keras_h5.py", str(npz), str(h5), "--offset", "4").returncode == 0
    r = _run("keras_h5_to_avse.py", str(h5), str(st))
    assert r.returncode == 0, r.stderr
    loaded = KerasModel.load(str(st))
    rng = np.random.default_rng(50)
    mel = rng.normal(-40, 12, (3, 80, 20)).astype(np.float32)
    video = rng.integers(0, 256, (3, 128, 128, 5)).astype(np.float32)
    ref = K.forward(m.layer_dict(), mel, video)
    dw = ops.DeviceWeights(loaded, dtype)
    got = ops.forward(dw, torch.from_numpy(mel).to(gpu), torch.from_numpy(video).to(gpu), checked=True).cpu().numpy()
    err = float(np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2)))
    print(f"HDF5 model, {dtype}: output RMS {np.sqrt(np.mean(ref ** 2)):.3g}, abs RMS err {err:.3e}")
    assert dw.last_range_bits == 0
    # the fp32 forward's bounds (tests/test_gpu_forward.py): absolute RMS 1e-4 (north star) and relative 1e-5
    assert err <= 1e-4, err
    assert err <= 1e-5 * float(np.sqrt(np.mean(ref ** 2))) + 1e-12, err
