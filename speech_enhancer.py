"""Command-line entry with the reference's invocation (python speech_enhancer.py -bd BASE preprocess|train|predict ...);
see audio-visual-speech-enhancement_amd/speech_enhancer.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import avse_pkg  # noqa: E402

avse_pkg.load()
from avse_amd.speech_enhancer import main  # noqa: E402

if __name__ == "__main__":
    main()
