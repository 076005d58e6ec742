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
    # the other reductions, a dst reduce, and bool leaves (sent as uint8, returned as bool)
    v = torch.tensor([rank + 1.0, 5.0 - rank])
    res["min"] = comm.reduce(v.clone(), "min").tolist()
    res["max"] = comm.reduce(v.clone(), "max").tolist()
    res["product"] = comm.reduce(v.clone(), "product").tolist()
    res["mean"] = comm.reduce(v.clone(), "mean").tolist()
    res["dst"] = comm.reduce(v.clone(), "sum", dst=0).tolist()
    b = torch.tensor([rank == 0, True, False])
    rb = comm.reduce({"b": b}, "max")["b"]
    res["bool_reduce"] = (str(rb.dtype), rb.tolist())
    sb = comm.stack(b, dst=1)
    res["bool_stack"] = (str(sb.dtype), sb.tolist())
    cb = comm.cat([b[:rank + 1]])[0]
    res["bool_cat"] = (str(cb.dtype), cb.tolist())
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
        assert res[r]["min"] == [1.0, 4.0] and res[r]["max"] == [2.0, 5.0]
        assert res[r]["product"] == [2.0, 20.0] and res[r]["mean"] == [1.5, 4.5]
        assert res[r]["bool_reduce"] == ("torch.bool", [True, True, False])
        assert res[r]["bool_stack"] == ("torch.bool", [[True, True, False], [False, True, False]])
        assert res[r]["bool_cat"] == ("torch.bool", [True, False, True])
    assert res[0]["dst"] == [3.0, 9.0]
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


def _loop_metrics(ranks, expectation):
    """The reference's own loop (trainer.py:207-238), for the closed form."""
    query2LH = dict()
    for h, r, t, L, H in ranks:
        query2LH[(h, r, t)] = (L, H)
    hit1, hit3, hit10, mr, mrr = 0.0, 0.0, 0.0, 0.0, 0.0
    for (L, H) in query2LH.values():
        if expectation:
            for rank in range(L, H):
                if rank <= 1:
                    hit1 += 1.0 / (H - L)
                if rank <= 3:
                    hit3 += 1.0 / (H - L)
                if rank <= 10:
                    hit10 += 1.0 / (H - L)
                mr += rank / (H - L)
                mrr += 1.0 / rank / (H - L)
        else:
            rank = H - 1
            hit1 += rank <= 1
            hit3 += rank <= 3
            hit10 += rank <= 10
            mr += rank
            mrr += 1.0 / rank
    n = len(ranks)
    return dict(Data=len(query2LH), Hit1=hit1 / n, Hit3=hit3 / n, Hit10=hit10 / n, MR=mr / n, MRR=mrr / n)


@pytest.mark.parametrize("expectation", [True, False])
def test_closed_form_metrics_match_the_loop(expectation):
    """rank_metrics' closed form (Hit@k counts, MR mean, harmonic-number MRR)
    equals the reference loop to 1e-12 on ragged (L, H) ranges — short and
    |E|-long ranges, duplicate (h, r, t) rows whose later (L, H) wins — and on
    the UMLS fixture's ranks."""
    from rnnlogic_amd.trainer import TrainerPredictor
    rng = np.random.default_rng(0)
    E = 40943
    rows = []
    for i in range(3000):
        L = int(rng.integers(1, 200)) if i % 3 else int(rng.integers(1, E))
        H = L + 1 + (int(rng.integers(0, 5)) if i % 2 else int(rng.integers(0, E + 1 - L)))
        rows.append([int(rng.integers(0, 50)), int(rng.integers(0, 4)), int(rng.integers(0, 50)), L, H])
    rows.append([1, 1, 1, 1, E + 1])  # target not a candidate
    got = TrainerPredictor.rank_metrics(rows, expectation)
    want = _loop_metrics(rows, expectation)
    assert got["Data"] == want["Data"]
    for k in ("Hit1", "Hit3", "Hit10", "MR", "MRR"):
        assert abs(got[k] - want[k]) <= 1e-12 * max(1.0, abs(want[k])), (k, got[k], want[k])
    assert TrainerPredictor.rank_metrics([], expectation)["Data"] == 0
