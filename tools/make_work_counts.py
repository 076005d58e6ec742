"""Writes tests/golden/<name>_work.json: the exact SURVEY §8(d) work counts
of a bench workload (the test split in TestDataset order, the committed train
graph, the bench's rule file), computed by the C oracle
(oracle/ground_oracle.c): F (frontier expansions), T (edge traversals),
P ((rule, destination) pairs) and C (candidates).  bench.py reads the files
for its algorithmic-bytes figures (FB15k-237: `value` and the EM Predictor
line; kinship: config 2; WN18RR: config 3), so the timed program never runs
oracle code; tests/test_oracle_c.py re-derives a prefix of each.

Usage: python tools/make_work_counts.py [--threads N] [FB15k-237 kinship wn18rr]
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

NAMES = {"FB15k-237": "fb15k237", "kinship": "kinship", "wn18rr": "wn18rr"}


def out_path(name):
    return os.path.join(REPO, "tests", "golden", "%s_work.json" % NAMES[name])


def workload(name="FB15k-237"):
    path = datasets.materialize(name)
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
        model.set_rules(datasets.rule_file(name))
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
    args = sys.argv[1:]
    threads = os.cpu_count() or 1
    if args[:1] == ["--threads"]:
        threads, args = int(args[1]), args[2:]
    for name in args or ["FB15k-237"]:
        graph, model, rows = workload(name)
        work, ncand = work_counts(graph, model, rows, threads)
        F, T, P = (int(x) for x in work.sum(0))
        k = min(2000, len(rows))
        rf = datasets.rule_file(name)
        res = {"workload": "%s test split (TestDataset order), %s train graph, %s" % (
                   name, "real" if name == "kinship" else "synthetic",
                   "rnnlogic_rules.txt" if "rnnlogic_rules" in rf else os.path.relpath(rf, REPO)),
               "queries": int(len(rows)), "rules": int(model.num_rules), "rows_sha256": rows_digest(rows),
               "F": F, "T": T, "P": P, "C": int(ncand.sum()),
               "prefix": {"queries": k, "F": int(work[:k, 0].sum()), "T": int(work[:k, 1].sum()),
                          "P": int(work[:k, 2].sum()), "C": int(ncand[:k].sum())}}
        with open(out_path(name), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))


if __name__ == "__main__":
    main()
