"""Import alias: `import tuplewise` loads the package directory
trade-offs-in-distributed-tuplewise-estimation-and-learning_amd/ (its name is not a Python
identifier, so it cannot be imported directly)."""
import importlib.util as _ilu
import pathlib as _pl
import sys as _sys

_DIR = _pl.Path(__file__).resolve().with_name(
    "trade-offs-in-distributed-tuplewise-estimation-and-learning_amd")
_spec = _ilu.spec_from_file_location(__name__, _DIR / "__init__.py",
                                     submodule_search_locations=[str(_DIR)])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
