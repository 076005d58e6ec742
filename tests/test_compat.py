"""The reference's entry scripts run on this package with their imports
unchanged: every name src/run_predictorplus.py:14-18 and
src/run_rnnlogic.py:14-19 import resolves through compat/ (top-level
`data`, `predictors`, ... bound to rnnlogic_amd's modules)."""
import ast
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(REPO, "compat")
REF_SRC = "/root/reference/src"

# (module, names) the two entry scripts import (the reference's API surface)
ENTRY_IMPORTS = [
    ("data", ["KnowledgeGraph", "TrainDataset", "ValidDataset", "TestDataset", "RuleDataset"]),
    ("predictors", ["Predictor", "PredictorPlus"]),
    ("generators", ["Generator"]),
    ("utils", ["load_config", "save_config", "set_logger", "set_seed"]),
    ("trainer", ["TrainerPredictor", "TrainerGenerator"]),
    ("comm", []),
    ("easydict", ["EasyDict"]),
    # imported by the reference's own modules (predictors.py / trainer.py)
    ("embedding", ["RotatE"]),
    ("layers", ["MLP", "FuncToNodeSum", "FuncToNode"]),
]


def _run(code):
    env = dict(os.environ, PYTHONPATH=COMPAT, PYTHONDONTWRITEBYTECODE="1")
    return subprocess.run([sys.executable, "-c", code], cwd="/tmp", env=env, capture_output=True, text=True,
                          timeout=300)


def test_entry_script_names_resolve():
    lines = []
    for mod, names in ENTRY_IMPORTS:
        lines.append("import %s" % mod if not names else "from %s import %s" % (mod, ", ".join(names)))
    # the top-level modules ARE the package's (shared state)
    lines.append("import rnnlogic_amd.comm, rnnlogic_amd.predictors, rnnlogic_amd.data")
    lines.append("assert comm is rnnlogic_amd.comm")
    lines.append("import predictors, data; assert predictors is rnnlogic_amd.predictors and data is rnnlogic_amd.data")
    lines.append("assert PredictorPlus.__module__ == 'rnnlogic_amd.predictors'")
    lines.append("cfg = EasyDict({'a': {'b': 1}}); assert cfg.a.b == 1")
    lines.append("print('ok')")
    p = _run("\n".join(lines))
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-2000:]


def _script_imports(path):
    """(module, [names]) of the top-level `from X import ...` / `import X`
    statements of a reference script whose module is one of the reference's
    own (the names this package must provide)."""
    own = {m for m, _ in ENTRY_IMPORTS}
    out = []
    for node in ast.parse(open(path).read()).body:
        if isinstance(node, ast.ImportFrom) and node.module in own:
            out.append((node.module, [a.name for a in node.names]))
        elif isinstance(node, ast.Import):
            out += [(a.name, []) for a in node.names if a.name in own]
    return out


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference mount absent (GPU box)")
@pytest.mark.parametrize("script", ["run_predictorplus.py", "run_rnnlogic.py"])
def test_reference_script_imports_resolve(script):
    """The import statements of the reference script itself (parsed, not
    copied) resolve through compat/."""
    imps = _script_imports(os.path.join(REF_SRC, script))
    assert imps, "no imports of the reference's modules found in %s" % script
    known = dict(ENTRY_IMPORTS)
    for mod, names in imps:
        assert set(names) <= set(known[mod]), (mod, names)
    code = "\n".join("import %s" % m if not n else "from %s import %s" % (m, ", ".join(n)) for m, n in imps)
    p = _run(code + "\nprint('ok')")
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-2000:]
