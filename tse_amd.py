"""Import shim for the engine package.

The package directory is ``tse-replication-package-1-million-fuzzing-sessions_amd/``
(the name the build contract asks for), which is not a valid Python identifier.
``import tse_amd`` loads that directory as a regular package named ``tse_amd``;
its submodules (``tse_amd.engine``, ``tse_amd.rq.rq1`` ...) then resolve normally.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "tse-replication-package-1-million-fuzzing-sessions_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
