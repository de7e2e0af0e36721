"""Host-side file plumbing of the preprocess / predict CLI (outside the hot path).

What is listed and where things go follows the reference's behaviour; the code is this build's own:

* corpus layout (reference dataset.py:10-49): ``<dataset>/<speaker>/audio/<clip>.wav`` with the clip's video at
  ``<dataset>/<speaker>/video/<clip>.<any extension>``; noise corpora are flat directories of wav files.
  `speech_clips` / `noise_files` return ``limit`` entries after an optional shuffle, like ``subset``.
* cache / output layout (reference speech_enhancer.py:91-184): ``<base>/cache/preprocessed/<data>``,
  ``<base>/cache/models/<model>/{model, normalization}``, ``<base>/out/<model>/<data>/<timestamp>/<speaker>/
  <clip>_<noise>/{source,noise,mixture,enhanced}.wav`` (+ .mp4 mux when ffmpeg exists).
"""
import random
import shutil
import subprocess
from collections import namedtuple
from datetime import datetime
from pathlib import Path

Clip = namedtuple("Clip", ["speaker_id", "audio_path", "video_path"])


def speakers(dataset_dir):
    """Speaker directories of the corpus (reference dataset.py:31-32)."""
    return sorted(p.name for p in Path(dataset_dir).iterdir() if p.is_dir())


def _video_for(audio_path):
    """The video file whose stem matches the wav's, under the speaker's video/ directory."""
    a = Path(audio_path)
    hits = sorted(a.parent.parent.joinpath("video").glob(a.stem + ".*"))
    if not hits:
        raise FileNotFoundError(f"no video for {audio_path}")
    return str(hits[0])


def speech_clips(dataset_dir, speaker_ids, limit=None, shuffle=False):
    clips = [Clip(spk, str(w), _video_for(w))
             for spk in speaker_ids for w in sorted(Path(dataset_dir, spk, "audio").glob("*.wav"))]
    if shuffle:
        random.shuffle(clips)
    return clips[:limit]


def noise_files(noise_dirs, limit=None, shuffle=False):
    files = [str(f) for d in noise_dirs for f in sorted(Path(d).iterdir())]
    if shuffle:
        random.shuffle(files)
    return files[:limit]


def pair_speech_with_noise(dataset_dir, speaker_ids, noise_dirs, limit=None, shuffle=True, augmentation_factor=1):
    """Speech clips zipped with noise files, both truncated to the shorter list (reference
    speech_enhancer.py:201-220: 4 clips + 1 noise file -> 1 pair); each augmentation round repeats the clips
    with the noise list re-drawn."""
    clips = speech_clips(dataset_dir, speaker_ids, limit, shuffle)
    noises = noise_files(noise_dirs, limit, shuffle)
    n = min(len(clips), len(noises))
    clips, noises = clips[:n], noises[:n]
    out_clips, out_noises = list(clips), list(noises)
    for _ in range(augmentation_factor - 1):
        out_clips += clips
        out_noises += random.sample(noises, n)
    return out_clips, out_noises


class Layout:
    """Paths under the CLI's base directory (directories are created on first use)."""

    def __init__(self, base_dir):
        self.base = Path(base_dir)

    def _dir(self, *parts):
        d = self.base.joinpath(*parts)
        d.mkdir(parents=True, exist_ok=True)
        return d

    def preprocessed(self, data_name):
        return str(self._dir("cache", "preprocessed") / (data_name + ".npz"))

    def model_dir(self, model_name):
        return self._dir("cache", "models", model_name)

    def model_file(self, model_name):
        return str(self.model_dir(model_name) / "model.safetensors")

    def keras_model_file(self, model_name):
        return str(self.model_dir(model_name) / "model.h5py")      # the reference's file (speech_enhancer.py:120-122)

    def normalizer_file(self, model_name):
        return str(self.model_dir(model_name) / "normalization.npz")

    def prediction_run_dir(self, model_name, data_name):
        """A fresh timestamped directory for one predict run."""
        d = self._dir("out", model_name, data_name) / "{:%Y-%m-%d_%H-%M-%S}".format(datetime.now())
        d.mkdir()
        return d


def write_prediction(run_dir, sample, enhanced_signal):
    """One sample's outputs: source / noise copies, the mixture and the enhanced speech as wav, and the two
    videos re-muxed with those tracks when ffmpeg is available and the video is a real video file."""
    d = Path(run_dir, sample.speaker_id,
             Path(sample.video_file_path).stem + "_" + Path(sample.noise_file_path).stem)
    d.mkdir(parents=True)
    shutil.copy2(sample.speech_file_path, d / "source.wav")
    shutil.copy2(sample.noise_file_path, d / "noise.wav")
    sample.mixed_signal.save_to_wav_file(str(d / "mixture.wav"))
    enhanced_signal.save_to_wav_file(str(d / "enhanced.wav"))
    ext = Path(sample.video_file_path).suffix
    if shutil.which("ffmpeg") and ext != ".npy":
        for name in ("mixture", "enhanced"):
            subprocess.run(["ffmpeg", "-y", "-loglevel", "error", "-i", sample.video_file_path, "-i",
                            str(d / (name + ".wav")), "-c:v", "copy", "-map", "0:v:0", "-map", "1:a:0",
                            str(d / (name + ext))], check=False)
    return str(d)
