"""Import shim: ``import kcmc_amd`` loads the package directory
``keypoint-consensus-motion-correction_amd/`` (a directory name Python cannot import
directly) under the name ``kcmc_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "keypoint-consensus-motion-correction_amd")
_spec = _ilu.spec_from_file_location("kcmc_amd", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["kcmc_amd"] = _mod
_spec.loader.exec_module(_mod)
