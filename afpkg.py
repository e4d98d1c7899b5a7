"""Registers the product package directory ``anchored-fusion_amd/`` under the importable
name ``anchored_fusion_amd`` (a hyphen is not a valid Python identifier).

Usage: ``import afpkg; import anchored_fusion_amd as af``.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "anchored-fusion_amd")
NAME = "anchored_fusion_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
