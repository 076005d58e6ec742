"""Per-step times of the PredictorPlus training step (bench.py's train_step
line: FB15k-237, B = 32, edge removal, RotatE feature, Adam) — diagnostic for
a per-shape first-use cost (GPU box).  Prints one line per step for:
  pass 1: batches 0..N-1 (each a new relation, so a new R_q rule count),
  pass 2: the same batches again (every shape seen once),
  pass 3: batches N..2N-1 with torch.backends.cudnn.enabled = False (torch's
          native LSTM instead of MIOpen's).
Usage: python tools/train_step_diag.py [N]"""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.data import DeviceTrainBatches  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev)
solver = TrainerPredictor(model, model.train_set, None, test_set, None, gpus=[0])
solver.optimizer = torch.optim.Adam(model.parameters(), lr=5e-3)
dtb = DeviceTrainBatches(model.train_set, dev)
model.train()
batches = [[x.unsqueeze(0) for x in dtb[i]] for i in range(2 * N)]


def run(label, bs):
    times = []
    for b in bs:
        torch.cuda.synchronize()
        t = time.perf_counter()
        solver.train_step(model, b, 0.2)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t) * 1e3)
    rq = [len(model.relation2rules[int(b[1][0, 0])]) for b in bs]
    print("%s: %s" % (label, " ".join("%.1f(R_q=%d)" % (t, q) for t, q in zip(times, rq))), flush=True)
    s = sorted(times)
    print("  median %.2f ms, min %.2f ms" % (s[len(s) // 2], s[0]), flush=True)


run("pass1 new shapes", batches[:N])
run("pass2 same shapes", batches[:N])
torch.backends.cudnn.enabled = False
run("pass3 cudnn off, new shapes", batches[N:2 * N])
run("pass4 cudnn off, same shapes", batches[N:2 * N])
