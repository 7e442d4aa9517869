"""Import helper for the `sift-features_amd/` package directory.

The package directory name carries a hyphen (the project's naming), so it is
registered as the importable module ``sift_features_amd`` by path.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "sift-features_amd")


def load():
    mod = sys.modules.get("sift_features_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "sift_features_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sift_features_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
