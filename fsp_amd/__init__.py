"""Import alias for the package directory
``few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd/``.

That directory name is not a valid Python identifier, so this shim points the
``fsp_amd`` package's search path at it and executes its ``__init__``.
``import fsp_amd.trainers.cocoop`` etc. then resolve inside the real package.
"""
import os as _os

_REAL = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd",
)
__path__ = [_REAL]
with open(_os.path.join(_REAL, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_REAL, "__init__.py"), "exec"))
