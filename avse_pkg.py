"""Import shim: registers the package directory `audio-visual-speech-enhancement_amd/` (not a valid
Python identifier) under the importable name `avse_amd`.

    import avse_pkg; avse = avse_pkg.load(); from avse_amd import ops
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "audio-visual-speech-enhancement_amd")
NAME = "avse_amd"


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
