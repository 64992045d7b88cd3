"""Import shim: the eraft_amd package lives in e-raft_amd/ (hyphenated directory, not a valid
identifier).  `import eraft_amd` loads e-raft_amd/__init__.py as the package `eraft_amd` and puts
it in sys.modules in place of this module, so `from eraft_amd.corr import CorrBlock` works too."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "e-raft_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
