"""Writes tests/golden/fb15k237_work.json: the exact SURVEY §8(d) work counts
of the bench workload (FB15k-237 test split in TestDataset order, committed
synthetic train graph, rnnlogic_rules.txt), computed by the C oracle
(oracle/ground_oracle.c): F (frontier expansions), T (edge traversals),
P ((rule, destination) pairs) and C (candidates).  bench.py reads the file for
its algorithmic-bytes figure, so the timed program never runs oracle code;
tests/test_oracle_c.py re-derives a prefix of it.

Usage: python tools/make_work_counts.py [threads]
"""
import contextlib
import hashlib
import json
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import ground_c  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "fb15k237_work.json")


def workload():
    path = datasets.materialize("FB15k-237")
    # bench.build_workload's order (run_predictorplus.py): seeds, graph, train/valid/test datasets
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    with contextlib.redirect_stdout(sys.stderr):
        graph = KnowledgeGraph(path)
        TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
        model = PredictorPlus(graph, type="emb", entity_feature="bias", aggregator="sum")
        model.set_rules(datasets.rule_file("FB15k-237"))
    rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
    return graph, model, rows


def work_counts(graph, model, rows, threads):
    cg = ground_c.CGraph(graph.entity_size, graph.relation_size, graph._train)
    orc = ground_c.Oracle(cg, model.rules, graph.relation_size)
    _, ncand, work = orc.digests(rows[:, 0], rows[:, 1], threads=threads, work=True)
    return work, ncand


def rows_digest(rows):
    return hashlib.sha256(np.ascontiguousarray(rows[:, :2], dtype=np.int64).tobytes()).hexdigest()


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    graph, model, rows = workload()
    work, ncand = work_counts(graph, model, rows, threads)
    F, T, P = (int(x) for x in work.sum(0))
    res = {"workload": "FB15k-237 test split (TestDataset order), synthetic train graph, rnnlogic_rules.txt",
           "queries": int(len(rows)), "rules": int(model.num_rules), "rows_sha256": rows_digest(rows),
           "F": F, "T": T, "P": P, "C": int(ncand.sum()),
           "prefix": {"queries": 2000, "F": int(work[:2000, 0].sum()), "T": int(work[:2000, 1].sum()),
                      "P": int(work[:2000, 2].sum()), "C": int(ncand[:2000].sum())}}
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
