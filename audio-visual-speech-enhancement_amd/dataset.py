"""Dataset listing with the semantics of /root/reference/dataset.py (host plumbing).

Layout: <base>/<speaker>/audio/<name>.wav with the mouth-crop video at <base>/<speaker>/video/<name>.*
(the reference decodes .mpg/.mp4 and crops with dlib; this build reads pre-cropped mouth stacks
saved as .npy [frames, 128, 128], see speech_enhancer.py).
"""
import glob
import os
import random
from collections import namedtuple

AudioVisualEntry = namedtuple("AudioVisualEntry", ["speaker_id", "audio_path", "video_path"])


class AudioVisualDataset:
    def __init__(self, base_path):
        self._base_path = base_path

    def subset(self, speaker_ids, max_files=None, shuffle=False):
        entries = []
        for speaker_id in speaker_ids:
            for audio_path in sorted(glob.glob(os.path.join(self._base_path, speaker_id, "audio", "*.wav"))):
                entries.append(AudioVisualEntry(speaker_id, audio_path, self._audio_to_video_path(audio_path)))
        if shuffle:
            random.shuffle(entries)
        return entries[:max_files]

    def list_speakers(self):
        return sorted(os.listdir(self._base_path))

    @staticmethod
    def _audio_to_video_path(audio_path):
        return glob.glob(os.path.splitext(audio_path.replace("audio", "video"))[0] + ".*")[0]


class AudioDataset:
    def __init__(self, base_paths):
        self._base_paths = base_paths

    def subset(self, max_files=None, shuffle=False):
        paths = [os.path.join(d, f) for d in self._base_paths for f in sorted(os.listdir(d))]
        if shuffle:
            random.shuffle(paths)
        return paths[:max_files]
