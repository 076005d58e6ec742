import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


class Fixture:
    """Reader for tests/golden/<case>.npz (written by tools/make_golden.py)."""

    def __init__(self, name):
        self.name = name
        self.z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.cfg = json.loads(str(self.z["cfg"]))
        self.sd = {k[3:]: self.z[k] for k in self.z.files if k.startswith("sd/")}
        self.ncalls = int(self.z["ncalls"])

    def call(self, k):
        p = "q%d/" % k
        g = lambda n: self.z[p + n]  # noqa: E731
        etr = g("etr")
        return dict(split=str(g("split")), index=int(g("index")), h=g("h"), r=g("r"), t=g("t"),
                    etr=etr if str(g("split")) == "train" else None, score=g("score"), mask=g("mask"),
                    coo=g("coo"))

    def dataset_path(self):
        from rnnlogic_amd import datasets
        return datasets.materialize(self.cfg["data"])

    def rule_path(self):
        from rnnlogic_amd import datasets
        return datasets.rule_file(self.cfg["data"])

    def rotate_path(self):
        from rnnlogic_amd import datasets
        emb = self.cfg.get("embedding")
        if not emb:
            return None
        if emb == "rotate":
            return datasets.rotate_path(self.cfg["data"])
        return datasets.rotate_path(self.cfg["data"], int(emb.split(":")[1]))


ALL_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN)
                   if f.endswith(".npz") and not f.startswith(("_", "train_", "pred_", "rules_", "eval_", "em_", "flow_")))
# reference miner rule pools (tools/make_golden_rules.py)
RULE_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("rules_") and f.endswith(".npz"))


def golden_rules(case):
    """[(head, body tuple)] of a tests/golden/rules_*.npz pool, reference order."""
    flat = np.load(os.path.join(GOLDEN, case + ".npz"))["flat"].astype(np.int64)
    rules, k = [], 0
    while k < len(flat):
        hd, ln = int(flat[k]), int(flat[k + 1])
        rules.append((hd, tuple(int(x) for x in flat[k + 2:k + 2 + ln])))
        k += 2 + ln
    return rules
# training-path fixtures (tools/make_golden_train.py)
TRAIN_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("train_") and f.endswith(".npz"))
TRAIN_SPECS = {  # dataset, PredictorPlus kwargs, RotatE dir — mirrors tools/make_golden_train.py CASES
    "train_umls_lstm_sum_bias": ("umls", dict(type="lstm", entity_feature="bias", aggregator="sum"), None),
    "train_umls_emb_pna_rotate": ("umls", dict(type="emb", entity_feature="RotatE", aggregator="pna"), 200),
    "train_kinship_lstm_sum_none": ("kinship", dict(type="lstm", entity_feature="none", aggregator="sum"), None),
    "train_kinship_emb_pna_bias": ("kinship", dict(type="emb", entity_feature="bias", aggregator="pna"), None),
    # the headline model (config 4): FB15k-237 lstm/sum + RotatE(D = 1000) trainable, edge removal
    "train_fb_lstm_sum_rotate": ("FB15k-237", dict(type="lstm", entity_feature="RotatE", aggregator="sum"), 1000),
}
# EM rule-weight Predictor fixtures (tools/make_golden_predictor.py)
PRED_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("pred_") and f.endswith(".npz"))
SMALL_CASES = [c for c in ALL_CASES if c.startswith(("umls", "kinship"))]


@pytest.fixture(scope="session")
def fixtures():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = Fixture(name)
        return cache[name]
    return get
