"""CPU tests of the host side: the C-ABI library loads and exports what include/avse.h declares,
the weight container / blob layout, persistence, and the mediaio stand-in.  No GPU compute."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "avse.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avse_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ["avse_ctx_create", "avse_spectrogram", "avse_weights_load", "avse_forward", "avse_mse",
              "avse_video_normalize", "avse_last_error", "avse_forward_profile"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    from avse_amd import _lib
    lib = _lib.load()
    for f in declared_functions():
        assert hasattr(lib, f), f"libavse.so does not export {f}"
        assert f in _lib.SIGNATURES, f"_lib.SIGNATURES lacks {f}"


def test_library_is_gfx950_code_object():
    from avse_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_spec640" in data and b"k_spec_seg" in data and b"k_conv" in data


def test_abi_version_and_blob_size():
    from avse_amd import _lib
    from avse_amd.model import blob_floats
    lib = _lib.load()
    assert lib.avse_abi_version() == _lib.ABI_VERSION == 3
    assert lib.avse_weights_blob_floats() == blob_floats()


def test_null_arguments_are_rejected_without_gpu_work():
    from avse_amd import _lib
    lib = _lib.load()
    rc = lib.avse_ctx_create(0, None)
    assert rc == 1 and b"NULL" in lib.avse_last_error()
    rc = lib.avse_forward(None, None, None, None, None, None, 1, None, None)
    assert rc == 1
    rc = lib.avse_forward_checked(None, None, None, None, None, None, 1, None, None, 0, None)
    assert rc == 1
    rc = lib.avse_range_status(None, None, None)
    assert rc == 1
    rc = lib.avse_weights_act_exponents(None, None, 0)
    assert rc == 1


def test_model_init_blob_roundtrip(tmp_path):
    from avse_amd.model import KerasModel, tensor_names
    m = KerasModel.init(seed=3, randomize=True)
    blob = m.to_blob()
    assert blob.dtype == np.float32 and blob.size == sum(int(np.prod(s)) for _, s in tensor_names())
    p = str(tmp_path / "model.h5py")
    m.save(p)
    m2 = KerasModel.load(p)
    assert np.array_equal(m2.to_blob(), blob)
    # Keras-default init: BN identity stats, zero bias
    d = KerasModel.init(seed=0).layer_dict()
    assert np.all(d["v_conv1_bn"]["gamma"] == 1) and np.all(d["v_conv1_bn"]["moving_variance"] == 1)
    assert np.all(d["enc_dense"]["bias"] == 0)


def test_keras_layouts():
    from avse_amd.model import KerasModel
    d = KerasModel.init(seed=0).layer_dict()
    assert d["a_conv1"]["kernel"].shape == (5, 5, 1, 64)
    assert d["v_conv1"]["kernel"].shape == (5, 5, 5, 128)
    assert d["enc_dense"]["kernel"].shape == (5248, 1312)
    assert d["d_deconv5"]["kernel"].shape == (5, 5, 64, 64)
    assert d["d_deconv6"]["kernel"].shape == (1, 1, 1, 64)
    assert d["dec_dense2_bn"]["gamma"].shape == (128,)
    # glorot limit respected
    lim = np.sqrt(6.0 / (5248 + 1312))
    assert np.abs(d["enc_dense"]["kernel"]).max() <= lim


def test_hdf5_is_rejected_with_a_clear_message(tmp_path):
    from avse_amd.model import KerasModel
    p = tmp_path / "model.h5py"
    p.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(ValueError, match="HDF5"):
        KerasModel.load(str(p))


def test_audio_signal_pad_truncate_in_place():
    from avse_amd.audio_io import AudioMixer, AudioSignal
    s = AudioSignal(np.arange(10, dtype=np.int16), 16000)
    s.pad_with_zeros(15)
    assert s.get_number_of_samples() == 15 and s.get_data(0)[-1] == 0
    s.truncate(4)
    assert s.get_data(0).tolist() == [0, 1, 2, 3]
    n = AudioSignal(np.ones(4), 16000)
    f = AudioMixer.snr_factor(s, n, snr_db=0)
    assert f == pytest.approx(np.sqrt(np.mean(np.arange(4.0) ** 2)))
    mix = AudioMixer.mix([s, n], [1, 1])
    assert mix.get_data(0).tolist() == [1, 2, 3, 4]


def test_wav_roundtrip(tmp_path):
    from avse_amd.audio_io import AudioSignal
    x = (np.sin(np.arange(1600) / 10) * 1000).astype(np.int16)
    p = str(tmp_path / "a.wav")
    AudioSignal(x, 16000).save_to_wav_file(p)
    y = AudioSignal.from_wav_file(p)
    assert y.get_sample_rate() == 16000 and np.array_equal(y.get_data(0), x)


def test_ops_refuse_cpu_tensors():
    import torch
    from avse_amd import ops
    with pytest.raises(TypeError):
        ops.spectrogram(torch.zeros(1, 3200))


def test_preprocessed_blob_and_normalizer_round_trip(tmp_path):
    """The CLI's caches are pickle-free: list[Sample] as one .npz (+ JSON metadata), the normaliser as .npz;
    both read back with allow_pickle=False."""
    from avse_amd import data_processor
    from avse_amd.audio_io import AudioSignal
    from avse_amd.speech_enhancer import Sample, load_preprocessed_blob, save_preprocessed_blob
    rng = np.random.default_rng(0)
    samples = []
    for i in range(3):
        n = 2 + i
        samples.append(Sample("spk%d" % i, "/v/%d.npy" % i, "/a/%d.wav" % i, "/n/%d.wav" % i,
                              rng.normal(size=(n, 128, 128, 5)).astype(np.float32),
                              rng.normal(size=(n, 80, 20)).astype(np.float32),
                              rng.normal(size=(n, 80, 20)).astype(np.float32),
                              rng.normal(size=(n, 80, 20)).astype(np.float32),
                              AudioSignal(rng.normal(size=3200 * n).astype(np.float32), 16000), 25.0 + i))
    p = str(tmp_path / "d.npz")
    save_preprocessed_blob(p, samples)
    got = load_preprocessed_blob(p)
    assert len(got) == 3
    for a, b in zip(samples, got):
        for f in ("speaker_id", "video_file_path", "speech_file_path", "noise_file_path", "video_frame_rate"):
            assert getattr(a, f) == getattr(b, f)
        for f in ("video_samples", "mixed_spectrograms", "speech_spectrograms", "noise_spectrograms"):
            assert np.array_equal(getattr(a, f), getattr(b, f))
        assert np.array_equal(a.mixed_signal.get_data(), b.mixed_signal.get_data())
        assert b.mixed_signal.get_sample_rate() == 16000
    norm = data_processor.VideoNormalizer(samples[0].video_samples)
    q = str(tmp_path / "normalization.npz")
    norm.save(q)
    back = data_processor.VideoNormalizer.load(q)
    assert np.array_equal(back.mean_image, norm.mean_image) and np.array_equal(back.std_image, norm.std_image)


def test_other_frame_rate_networks_build_and_bad_shapes_are_refused():
    """At 29.97 / 30 fps the reference slices [80, 24] spectrograms (data_processor.py:44-52) with 5 / 6 video frames
    per slice (:24), and Keras builds the matching network (concat 5888 -> Dense 1472, network.py:53-55; graphs
    pinned in tests/golden/network_spec_*fps.json).  build() makes those; the C library sizes their weight blobs
    the same way; shapes whose decoder cannot give back 80 x T (T not a multiple of 4) are refused up front."""
    from avse_amd import _lib
    from avse_amd.model import blob_floats
    from avse_amd.network import SpeechEnhancementNetwork
    lib = _lib.load()
    for T, F in [(20, 5), (24, 5), (24, 6), (8, 1)]:
        assert lib.avse_weights_blob_floats_shape(T, F) == blob_floats(T, F), (T, F)
    net = SpeechEnhancementNetwork.build((80, 24), (128, 128, 6))
    assert (net.model.T, net.model.F) == (24, 6)
    assert net.model.tensors["enc_dense/kernel"].shape == (5888, 1472)
    assert net.model.tensors["dec_dense2/kernel"].shape == (1472, 3840)
    assert lib.avse_weights_blob_floats_shape(22, 5) == -1 and lib.avse_weights_blob_floats_shape(24, 9) == -1
    with pytest.raises(NotImplementedError):
        SpeechEnhancementNetwork.build((80, 22), (128, 128, 5))
    with pytest.raises(NotImplementedError):
        SpeechEnhancementNetwork.build((80, 20), (64, 64, 5))


def _checked_harness():
    """tests/native/abi_checked (csrc/Makefile `checked`: the checked build + host AddressSanitizer); built here when
    missing (make is incremental; __graft_entry__.build() builds it too)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "native", "abi_checked")
    csrc = os.path.join(ROOT, "audio-visual-speech-enhancement_amd", "csrc")
    subprocess.check_call(["make", "-C", csrc, "-j8", "checked"], stdout=subprocess.DEVNULL)
    return exe


def test_checked_build_harness_host_part():
    """The C-ABI's host paths (argument validation, blob sizes, shape refusals) under AddressSanitizer; without a
    GPU the harness stops after them (tests/test_gpu_checked.py runs the device part)."""
    import subprocess
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([_checked_harness()], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 0 failure(s)" in r.stdout


def test_release_and_checked_build_flags():
    from avse_amd import _lib
    assert _lib.load().avse_build_flags() == (1 if "debug" in os.path.basename(_lib.LIB_PATH) else 0)


def test_predict_rank_command_threads_argv():
    """`predict -g N` relaunches the reference-shaped entry script with the arguments main() parsed (it used
    sys.argv, wrong for main(argv) and for module invocations)."""
    import os
    from avse_amd import speech_enhancer as se
    argv = ["-bd", "/tmp/base", "predict", "-mn", "m", "-dn", "d", "-g", "2"]
    cmd = se.rank_command(2, argv, 12345)
    assert cmd[cmd.index("--nproc-per-node=2")] and "--master-port" in cmd and cmd[cmd.index("--master-port") + 1] == "12345"
    i = cmd.index(se.ENTRY_SCRIPT)
    assert cmd[i + 1:] == argv
    assert os.path.isfile(se.ENTRY_SCRIPT) and os.path.basename(se.ENTRY_SCRIPT) == "speech_enhancer.py"


def test_forward_is_asynchronous_by_default_and_the_reference_api_checks():
    """ops.forward stays the asynchronous, capturable avse_forward unless a caller opts in; the synchronous
    reference-shaped API (SpeechEnhancementNetwork.predict_device / predict / evaluate) opts in for split weights."""
    import inspect
    from avse_amd import network, ops
    assert inspect.signature(ops.forward).parameters["checked"].default is False
    assert inspect.signature(network.SpeechEnhancementNetwork.predict_device).parameters["checked"].default is None


def test_range_set_aside_keeps_earlier_bits():
    """Context.set_aside_range moves the device word's bits to the host side; range_status still returns them once."""
    from avse_amd import _lib

    class Fake(_lib.Context):
        def __init__(self):
            self._set_aside, self.words = 0, [0x40, 0x2, 0]

        def _read_range(self, stream):
            return self.words.pop(0)

    c = Fake()
    c.set_aside_range()
    assert c.range_status() == 0x42 and c.range_status() == 0


def test_concat_exponent_mismatch_is_flagged_at_load():
    """a_conv5 / v_conv6 share the smaller activation exponent; a model whose halves want different ones is
    flagged when float32_split weights are built (the rule restated from csrc/capi.hip act_exponents)."""
    import warnings
    from avse_amd import ops
    from avse_amd.model import KerasModel
    m = KerasModel.init(seed=3, randomize=True)
    assert ops.act_exponent(m, "a_conv5") == ops.act_exponent(m, "v_conv6") == 0
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        ops._warn_concat_exponents(m)
    for p in ("gamma", "beta"):
        m.tensors["v_conv6_bn/" + p] = (m.tensors["v_conv6_bn/" + p] * np.float32(2.0 ** -14)).astype(np.float32)
    assert ops.act_exponent(m, "v_conv6") >= 14
    with pytest.warns(RuntimeWarning, match="video half"):
        ops._warn_concat_exponents(m)
