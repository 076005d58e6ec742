"""Run a script against an A/B build of the library (tools/build_variants.sh):
    python tools/ab_run.py rnnlogic_amd/_build/variants/a.so bench.py --feature bias ...
Diagnostic only: the product loader (rnnlogic_amd/_native.py) always loads
rnnlogic_amd/_build/librnnlogic_hip.so; this sets its LIB_PATH before the
first load and then runs the script as __main__."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from rnnlogic_amd import _native  # noqa: E402

lib, script = os.path.abspath(sys.argv[1]), sys.argv[2]
if not os.path.exists(lib):
    sys.exit("ab_run: no library %s" % lib)
_native.LIB_PATH = lib
sys.argv = [script] + sys.argv[3:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
