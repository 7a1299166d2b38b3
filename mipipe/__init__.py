"""Importable alias for the `distributed-llm-pipeline_amd/` package directory.

The framework's package directory is `distributed-llm-pipeline_amd/` (a name with hyphens, not a
valid Python identifier); this shim registers it under the import name `mipipe`, so
`import mipipe.ops`, `from mipipe.models import ...` etc. resolve to the files in that directory.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                     "distributed-llm-pipeline_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
