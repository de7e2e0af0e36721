"""MI355X-native (gfx950) hot path of melspectrum007/audio-visual-speech-enhancement.

The directory name contains hyphens, so the package is imported under the name `avse_amd`
(see avse_pkg.py at the repository root).

Modules
  ops             device-level entry points over libavse.so (include/avse.h)
  data_processor  reference-shaped audio front end (data_processor.py)
  network         SpeechEnhancementNetwork (network.py)
  model           Keras-layout parameter container / weight blob
  parallel        clip sharding across ranks + RCCL gather
  speech_enhancer the preprocess / predict CLI (speech_enhancer.py)
"""
from . import _lib  # noqa: F401
from .model import KerasModel, LAYERS  # noqa: F401
