"""Import alias for the package directory ``causal-unified-language-vision_amd/``.

The directory name required by the repository layout is not a valid Python identifier, so
``import cullavo_amd`` executes this file, which loads that directory as the package
``cullavo_amd`` (submodules resolve through its ``__path__``) and replaces itself in
``sys.modules``.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "causal-unified-language-vision_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
