"""Host side of the trainer mirror (CPU): the ranking / metric code against the
reference's own evaluate() numbers, and the multi-process path (gloo,
world size 2): comm.reduce/stack/cat and a sharded TrainerPredictor.evaluate
whose gathered ranks reproduce the single-process result."""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import Fixture

CASE = "umls_lstm_sum_bias"  # every test batch of the split is in this fixture


class GoldenScores(torch.nn.Module):
    """Stand-in predictor returning the reference's own scores per batch."""

    def __init__(self, fx):
        super(GoldenScores, self).__init__()
        self.table = {}
        for k in range(fx.ncalls):
            c = fx.call(k)
            if c["split"] == "test":
                self.table[(int(c["r"][0]),) + tuple(int(x) for x in c["h"])] = (c["score"], c["mask"])
        self.num_rules = 1
        self.dummy = torch.nn.Parameter(torch.zeros(1))

    def forward(self, all_h, all_r, edges_to_remove):
        s, m = self.table[(int(all_r[0]),) + tuple(int(x) for x in all_h)]
        return torch.from_numpy(s), torch.from_numpy(m)


def _setup():
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    fx = Fixture(CASE)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    graph = KnowledgeGraph(datasets.materialize(fx.cfg["data"]))
    train_set = TrainDataset(graph, 32)
    valid_set = ValidDataset(graph, 32)
    test_set = TestDataset(graph, 32)
    return fx, train_set, valid_set, test_set


def test_evaluate_reproduces_reference_metrics():
    from rnnlogic_amd.trainer import TrainerPredictor
    fx, train_set, valid_set, test_set = _setup()
    solver = TrainerPredictor(GoldenScores(fx), train_set, valid_set, test_set, None, gpus=None)
    mrr = solver.evaluate("test", expectation=True)
    assert abs(mrr - float(fx.z["eval/mrr"])) < 1e-12
    # the other metrics through the same code path
    ranks = []
    for batch in torch.utils.data.DataLoader(test_set, 1):
        h, r, t, flag = [x.squeeze(0) for x in batch]
        s, m = solver.model(h, r, None)
        L, H = TrainerPredictor.filtered_ranks(s, m, flag, t, test_set.graph.entity_size)
        ranks += torch.stack([h, r, t, L, H], 1).tolist()
    m = TrainerPredictor.rank_metrics(ranks, True)
    for key in ("Hit1", "Hit3", "Hit10", "MR"):
        assert abs(m[key] - float(fx.z["eval/" + key])) <= 5e-7, key


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from rnnlogic_amd import comm
    from rnnlogic_amd.trainer import TrainerPredictor
    comm.init_process_group("gloo", init_method="env://")
    res = {}
    # reduce / stack / cat on a nested structure, ragged dim 0 for cat
    x = {"a": torch.full((3,), float(rank + 1)), "b": [torch.arange(rank + 2, dtype=torch.long)]}
    red = comm.reduce({"a": x["a"].clone()})
    res["reduce"] = red["a"].tolist()
    st = comm.stack(x["a"])
    res["stack"] = st.tolist()
    ct = comm.cat(x)
    res["cat_a"] = ct["a"].tolist()
    res["cat_b"] = ct["b"][0].tolist()
    # sharded evaluate
    fx, train_set, valid_set, test_set = _setup()
    solver = TrainerPredictor(GoldenScores(fx), train_set, valid_set, test_set, None, gpus=None)
    res["mrr"] = solver.evaluate("test", expectation=True)
    comm.synchronize()
    torch.save(res, os.path.join(out_dir, "rank%d.pt" % rank))
    torch.distributed.destroy_process_group()


def test_gloo_world2_comm_and_sharded_evaluate(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    res = [torch.load(os.path.join(str(tmp_path), "rank%d.pt" % r), weights_only=True) for r in range(world)]
    for r in range(world):
        assert res[r]["reduce"] == [3.0, 3.0, 3.0]
        assert res[r]["stack"] == [[1.0] * 3, [2.0] * 3]
        assert res[r]["cat_a"] == [1.0] * 3 + [2.0] * 3
        assert res[r]["cat_b"] == [0, 1] + [0, 1, 2]
    # both ranks agree; the gathered ranks (padding duplicates included) give
    # the reference's formula over the padded shard union
    assert res[0]["mrr"] == res[1]["mrr"]
    from rnnlogic_amd.trainer import TrainerPredictor
    fx, train_set, valid_set, test_set = _setup()
    model = GoldenScores(fx)
    ranks = []
    for rank in range(world):
        sampler = torch.utils.data.DistributedSampler(test_set, world, rank)
        for idx in sampler:
            h, r, t, flag = test_set[idx]
            s, m = model(h, r, None)
            L, H = TrainerPredictor.filtered_ranks(s, m, flag, t, test_set.graph.entity_size)
            ranks += torch.stack([h, r, t, L, H], 1).tolist()
    want = TrainerPredictor.rank_metrics(ranks, True)["MRR"]
    assert abs(res[0]["mrr"] - want) < 1e-12
    if len(test_set) % world == 0:
        assert abs(res[0]["mrr"] - float(fx.z["eval/mrr"])) < 1e-12
