"""Import helper: the package directory name (open-vocabulary-3d-object-detection_amd)
is not a Python identifier, so it is registered as ``ov3d_amd``."""
import importlib.util
import os
import sys

PKG_NAME = "ov3d_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "open-vocabulary-3d-object-detection_amd")


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(PKG_NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
