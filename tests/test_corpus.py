"""Host plumbing of the CLI (corpus.py): corpus listing and pairing semantics of the reference
(dataset.py:10-49, speech_enhancer.py:188-220) on a temporary directory tree; no GPU."""
import os
import types

from avse_amd import corpus
from avse_amd.speech_enhancer import selected_speakers


def make_tree(tmp):
    ds = tmp / "ds"
    for spk in ("s1", "s2", "s3"):
        (ds / spk / "audio").mkdir(parents=True)
        (ds / spk / "video").mkdir(parents=True)
        for clip in ("a", "b"):
            (ds / spk / "audio" / (clip + ".wav")).write_bytes(b"")
            (ds / spk / "video" / (clip + ".mpg")).write_bytes(b"")
    noise = tmp / "noise"
    noise.mkdir()
    (noise / "n1.wav").write_bytes(b"")
    return ds, noise


def test_listing_and_pairing(tmp_path):
    ds, noise = make_tree(tmp_path)
    assert corpus.speakers(ds) == ["s1", "s2", "s3"]
    clips = corpus.speech_clips(ds, ["s1", "s2"])
    assert [(c.speaker_id, os.path.basename(c.audio_path), os.path.basename(c.video_path)) for c in clips] == \
        [("s1", "a.wav", "a.mpg"), ("s1", "b.wav", "b.mpg"), ("s2", "a.wav", "a.mpg"), ("s2", "b.wav", "b.mpg")]
    assert len(corpus.speech_clips(ds, ["s1", "s2"], limit=3, shuffle=True)) == 3
    # 4 clips x 1 noise file -> one pair (speech_enhancer.py:208 zips to the shorter list)
    sp, nz = corpus.pair_speech_with_noise(ds, ["s1", "s2"], [noise], limit=1000)
    assert len(sp) == len(nz) == 1
    sp, nz = corpus.pair_speech_with_noise(ds, ["s1"], [noise], augmentation_factor=3)
    assert len(sp) == len(nz) == 3


def test_selected_speakers(tmp_path):
    ds, _ = make_tree(tmp_path)
    args = types.SimpleNamespace(dataset_dir=str(ds), speakers=None, ignored_speakers=["s2"])
    assert selected_speakers(args) == ["s1", "s3"]
    args = types.SimpleNamespace(dataset_dir=str(ds), speakers=["s3", "s1"], ignored_speakers=None)
    assert selected_speakers(args) == ["s3", "s1"]


def test_layout_and_output(tmp_path):
    from collections import namedtuple
    lay = corpus.Layout(tmp_path / "base")
    assert lay.preprocessed("d").endswith(os.path.join("cache", "preprocessed", "d.npz"))
    assert lay.model_file("m").endswith(os.path.join("cache", "models", "m", "model.safetensors"))
    run = lay.prediction_run_dir("m", "d")
    (tmp_path / "s.wav").write_bytes(b"S")
    (tmp_path / "n.wav").write_bytes(b"N")

    class Sig:
        def save_to_wav_file(self, p):
            open(p, "wb").write(b"W")

    S = namedtuple("S", "speaker_id video_file_path noise_file_path speech_file_path mixed_signal")
    d = corpus.write_prediction(run, S("s1", "/x/clip.npy", str(tmp_path / "n.wav"), str(tmp_path / "s.wav"), Sig()),
                                Sig())
    assert sorted(os.listdir(d)) == ["enhanced.wav", "mixture.wav", "noise.wav", "source.wav"]
    assert os.path.basename(d) == "clip_n"
