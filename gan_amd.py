"""Import shim: the package directory is named ``-gan-_amd`` (not a Python identifier).

``import gan_amd`` loads ``-gan-_amd/__init__.py`` as the package ``gan_amd`` and replaces this
shim module with it, so ``import gan_amd.ops`` etc. work.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "-gan-_amd")
_spec = importlib.util.spec_from_file_location("gan_amd", os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["gan_amd"] = _mod
_spec.loader.exec_module(_mod)
