"""Top-level `embedding` for the reference's entry scripts (src/run_predictorplus.py,
src/run_rnnlogic.py import `embedding` as a top-level module): this module IS
rnnlogic_amd.embedding — the import binds the package module itself, so module state
(e.g. comm's process groups) is shared with code importing the package."""
import importlib
import os
import sys

try:
    importlib.import_module("rnnlogic_amd")
except ImportError:  # compat/ on sys.path without the repo root
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.modules[__name__] = importlib.import_module("rnnlogic_amd.embedding")
