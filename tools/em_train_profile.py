"""Host profile of the EM loop's predictor training (TrainerPredictor.train
with Predictor(bias), FB15k-237, rnnlogic_rules.txt): cProfile over 300
batches plus torch.profiler's sync count (diagnostic; GPU box).
Usage: python tools/em_train_profile.py"""
import contextlib
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import Predictor  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402
from rnnlogic_amd.utils import set_seed  # noqa: E402

with contextlib.redirect_stdout(sys.stderr):
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize("FB15k-237"))
    train_set = TrainDataset(graph, 32)
    valid_set = ValidDataset(graph, 32)
    test_set = TestDataset(graph, 32)
    predictor = Predictor(graph, entity_feature="bias")
    predictor.set_rules(datasets.rule_file("FB15k-237"))
optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
solver = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[0])
with contextlib.redirect_stdout(sys.stderr):
    solver.train(batch_per_epoch=20, smoothing=0.2, print_every=1000)
torch.cuda.synchronize()
t = time.perf_counter()
with contextlib.redirect_stdout(sys.stderr):
    solver.train(batch_per_epoch=300, smoothing=0.2, print_every=1000)
torch.cuda.synchronize()
print("ms per batch: %.3f" % ((time.perf_counter() - t) / 300 * 1e3))
pr = cProfile.Profile()
pr.enable()
with contextlib.redirect_stdout(sys.stderr):
    solver.train(batch_per_epoch=300, smoothing=0.2, print_every=1000)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts) as prof:
    with contextlib.redirect_stdout(sys.stderr):
        solver.train(batch_per_epoch=50, smoothing=0.2, print_every=1000)
    torch.cuda.synchronize()
ka = prof.key_averages()
print(ka.table(sort_by="self_cuda_time_total", row_limit=25, max_name_column_width=55))
print(ka.table(sort_by="count", row_limit=40, max_name_column_width=55))
