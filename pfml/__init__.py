"""Importable name of the framework package.

The package sources live in the directory
``jkmp22-machine-learning-and-the-implementable-efficient-frontier-replication_amd/``
(a name that is not a Python identifier).  This stub makes ``pfml`` a package whose
``__path__`` *is* that directory, so every submodule is imported exactly once, as
``pfml.<sub>``.
"""
import os as _os

PACKAGE_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "jkmp22-machine-learning-and-the-implementable-efficient-frontier-replication_amd",
)
__path__ = [PACKAGE_DIR]

with open(_os.path.join(PACKAGE_DIR, "__init__.py"), encoding="utf-8") as _f:
    exec(compile(_f.read(), _os.path.join(PACKAGE_DIR, "__init__.py"), "exec"))
