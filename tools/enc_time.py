"""Time the HIP LSTM rule encoder on the FB15k-237 bench model's 131,883
rules (diagnostic; GPU box) and check it against torch's LSTM:
python tools/enc_time.py (an A/B build: python tools/ab_run.py <lib.so> tools/enc_time.py)."""
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
with torch.no_grad():
    ms = bench.time_forward(lambda: model._encode_rules_hip(dev), 20) * 1e3
    got = model._encode_rules_hip(dev)
    want = model.encode_rules(model.rule_features.to(dev))
print("%s encoder %.3f ms, max |hip - torch| %.2e" % (os.path.basename(__import__("rnnlogic_amd._native")._native.LIB_PATH), ms,
                                                      (got - want).abs().max().item()))
