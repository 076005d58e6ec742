"""bench.py's multi-GPU split (CPU): the rows each rank times are the
reference evaluate()'s DistributedSampler shard of the test batches
(src/trainer.py:150) — shards cover every batch, ranks hold equal batch
counts, and the only repeats are the sampler's padding (len % world)."""
import collections
import random

import numpy as np
import pytest
import torch


def _test_set(data):
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    graph = KnowledgeGraph(datasets.materialize(data))
    TrainDataset(graph, 32)
    ValidDataset(graph, 32)
    return TestDataset(graph, 32)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_partition_the_split(world):
    import bench
    ts = _test_set("umls")
    nb = len(ts)
    shards = [bench.shard_rows(ts, world, rank) for rank in range(world)]
    per_rank = -(-nb // world)
    seen = collections.Counter()
    for rows, idx in shards:
        assert len(idx) == per_rank
        assert rows.shape == (sum(len(ts.batches[i]) for i in idx), 3)
        np.testing.assert_array_equal(rows, np.asarray([x for i in idx for x in ts.batches[i]]).reshape(-1, 3))
        seen.update(idx)
    assert set(seen) == set(range(nb))
    dup = sum(c - 1 for c in seen.values())
    assert dup == per_rank * world - nb
    # same order as the reference's sampler on that rank
    for rank, (_, idx) in enumerate(shards):
        want = list(iter(torch.utils.data.DistributedSampler(ts, world, rank)))
        assert idx == want
