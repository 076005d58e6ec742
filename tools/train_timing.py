"""Wall time per batch of TrainerPredictor.train on FB15k-237 (diagnostic; GPU
box): the bench model (PredictorPlus(lstm, sum) + RotatE D = 1000) and the
final PredictorPlus stage of run_rnnlogic.py (emb, sum, bias), each with the
training lookahead on (prefetch_depth 2, the default) and off (0).
Usage: python tools/train_timing.py [n_batches] [profile]
`profile`: torch.profiler over one train() call of each model (depth 2)
instead, top ops by host time."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 200
prof = len(sys.argv) > 2 and sys.argv[2] == "profile"
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, rot_model, rows = bench.build_workload("RotatE")
    train_set = rot_model.train_set
    emb_model = PredictorPlus(graph, hidden_dim=16)
    emb_model.set_rules(bench.datasets.rule_file("FB15k-237"))
for name, model in (("emb_sum_bias", emb_model), ("lstm_sum_rotate", rot_model)):
    model = model.to(dev)
    if prof:
        model.prefetch_depth = 2
        opt = torch.optim.Adam(model.parameters(), lr=5e-3)
        solver = TrainerPredictor(model, train_set, None, test_set, opt, gpus=[0])
        solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
        torch.cuda.synchronize()
        acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
        with torch.profiler.profile(activities=acts) as p:
            solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
            torch.cuda.synchronize()
        print("== %s, %d batches" % (name, nb))
        print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=60))
        continue
    for depth in (2, 0):
        model.prefetch_depth = depth
        opt = torch.optim.Adam(model.parameters(), lr=5e-3)
        solver = TrainerPredictor(model, train_set, None, test_set, opt, gpus=[0])
        solver.train(batch_per_epoch=20, smoothing=0.2, print_every=10 ** 9)  # warm-up (shapes, tables)
        torch.cuda.synchronize()
        t = time.perf_counter()
        solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / nb
        t = time.perf_counter()
        train_set.make_batches()  # once per train() call (the epoch's shuffle, host)
        mb = (time.perf_counter() - t) * 1e3
        print("%s prefetch_depth %d: %.3f ms per batch over %d batches, %.3f without the epoch shuffle "
              "(make_batches %.1f ms; dropped lookaheads %d)"
              % (name, depth, ms, nb, ms - mb / nb, mb, getattr(model, "prefetch_dropped", 0)), flush=True)
