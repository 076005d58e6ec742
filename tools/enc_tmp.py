import os, sys, contextlib, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
with torch.no_grad():
    ms = bench.time_forward(lambda: model._encode_rules_hip(dev), 20) * 1e3
print("%s encoder %.3f ms" % (os.environ.get("V"), ms))
