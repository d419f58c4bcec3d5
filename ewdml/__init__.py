"""Import name for the framework.

The source tree lives in ``efficient-workers-in-distributed-machine-learning_amd/`` (a directory
name that is not a valid Python identifier).  This shim makes that directory the package path of
``ewdml`` and executes its ``__init__``, so ``import ewdml`` / ``from ewdml.models import ...``
resolve to the real sources without copying or installing anything.
"""
import os as _os

_ROOT = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "efficient-workers-in-distributed-machine-learning_amd",
)
__path__ = [_ROOT]  # noqa: F821 - submodules are found in the real source directory
__file__ = _os.path.join(_ROOT, "__init__.py")

with open(__file__, "r", encoding="utf-8") as _f:
    exec(compile(_f.read(), __file__, "exec"))  # noqa: S102 - our own package init
