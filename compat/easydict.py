"""`easydict` for the reference's entry scripts on images without the
package (src/run_predictorplus.py / run_rnnlogic.py import EasyDict at the
top; neither this image nor the GPU box has it).  When an installed
easydict exists further down sys.path it is loaded instead, so this module
only stands in for a missing one."""
import importlib.machinery
import importlib.util
import os
import sys

_here = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.machinery.PathFinder.find_spec(
    "easydict", [p for p in sys.path if os.path.abspath(p or ".") != _here])
if _spec is not None:
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules[__name__] = _mod
    _spec.loader.exec_module(_mod)
else:
    try:
        importlib.import_module("rnnlogic_amd")
    except ImportError:
        sys.path.insert(0, os.path.dirname(_here))
    from rnnlogic_amd.utils import EasyDict  # noqa: F401
