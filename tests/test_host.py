"""CPU-only tests of the host side: the C-ABI library loads and exports every
declared symbol, argument validation works without a GPU, and the Python
mirror of the reference API (data/predictors/layers) reproduces the
reference's batches, parameter names/shapes and seeded initialisation."""
import os
import random
import re

import numpy as np
import pytest
import torch

from conftest import REPO, SMALL_CASES

HEADER = os.path.join(REPO, "include", "rnnlogic_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rnnl_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from rnnlogic_amd import _native
    L = _native.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(n for n, _, _ in _native.SIGNATURES) == syms


def test_argument_validation_without_gpu():
    import ctypes
    from rnnlogic_amd import _native
    L = _native.lib()
    h = ctypes.c_void_p()
    assert L.rnnl_graph_create(None, 3, 5, 2, ctypes.byref(h)) == _native.RNNL_ERR_INVALID
    assert b"bad arguments" in L.rnnl_last_error()
    bad = np.asarray([[0, 5, 1]], dtype=np.int32)  # relation out of range
    assert L.rnnl_graph_create(bad.ctypes.data_as(ctypes.c_void_p), 1, 4, 2, ctypes.byref(h)) == 1
    assert b"out of range" in L.rnnl_last_error()
    assert L.rnnl_forward_workspace_size(None, None, 1, 1, None) == _native.RNNL_ERR_INVALID


def test_missing_library_fails_loudly(monkeypatch):
    from rnnlogic_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/librnnlogic_hip.so")
    with pytest.raises(RuntimeError, match="missing"):
        _native.lib()


@pytest.mark.parametrize("case", SMALL_CASES)
def test_datasets_reproduce_reference_batches(case, fixtures):
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    fx = fixtures(case)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    g = KnowledgeGraph(fx.dataset_path())
    tr = TrainDataset(g, 32)
    ValidDataset(g, 32)
    te = TestDataset(g, 32)
    flat = np.asarray([x for b in te.batches for x in b], dtype=np.int64)
    np.testing.assert_array_equal(flat, fx.z["batches"])
    import hashlib
    trb = np.asarray([x for b in tr.batches for x in b], dtype=np.int64)
    assert hashlib.sha256(trb.tobytes()).hexdigest() == str(fx.z["train_sha"])
    # items: train batch edge ids index the reference's relation-local edge table
    all_h, all_r, all_t, target, etr = tr[0]
    heads = g.relation2adjacency[int(all_r[0])][0][1]
    tails = g.relation2adjacency[int(all_r[0])][0][0]
    assert torch.equal(heads[etr], all_h) and torch.equal(tails[etr], all_t)
    assert target.sum() >= len(all_h)


@pytest.mark.parametrize("case", SMALL_CASES)
def test_predictorplus_state_dict_and_seeded_init(case, fixtures):
    """Same module tree as the reference: identical keys/shapes, and a seeded
    construction reproduces the reference's initial parameters bit for bit."""
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.predictors import PredictorPlus
    fx = fixtures(case)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    g = KnowledgeGraph(fx.dataset_path())
    TrainDataset(g, 32)
    ValidDataset(g, 32)
    TestDataset(g, 32)
    m = PredictorPlus(g, embedding_path=fx.rotate_path(), **fx.cfg["model"])
    m.set_rules(fx.rule_path())
    sd = m.state_dict()
    keys = sorted(k for k in sd if not k.startswith("RotatE."))
    assert keys == sorted(fx.sd)
    for k in keys:
        assert tuple(sd[k].shape) == fx.sd[k].shape, k
        np.testing.assert_array_equal(sd[k].numpy(), fx.sd[k], err_msg=k)


def test_grounding_api_needs_gpu(fixtures):
    """KnowledgeGraph.grounding is the HIP grounding (no CPU path): CPU
    inputs raise.  Its counts are checked on the GPU in
    tests/test_gpu_graph_api.py."""
    from rnnlogic_amd.data import KnowledgeGraph
    fx = fixtures("umls_lstm_sum_bias")
    g = KnowledgeGraph(fx.dataset_path())
    with pytest.raises(RuntimeError, match="HIP path"):
        g.grounding(torch.zeros(2, dtype=torch.int64), 0, [1, 2], None)


def test_device_train_batches_tables():
    """The key tables behind data.DeviceTrainBatches (built on the host,
    uploaded once): hr2o CSR and the relation-local edge id map."""
    import numpy as np
    import torch
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import DeviceTrainBatches, KnowledgeGraph, TrainDataset
    graph = KnowledgeGraph(datasets.materialize("umls"))
    db = DeviceTrainBatches(TrainDataset(graph, 32), torch.device("cpu"))
    keys, offs, vals = db.hr2o.keys.numpy(), db.hr2o.offs.numpy(), db.hr2o.vals.numpy()
    assert (np.diff(keys) > 0).all() and len(offs) == len(keys) + 1
    E = graph.entity_size
    for h, r, t in graph.train_facts[::97]:
        i = np.searchsorted(keys, r * E + h)
        assert keys[i] == r * E + h
        assert list(vals[offs[i]:offs[i + 1]]) == graph.hr2o[graph.encode_hr(h, r)]
        j = np.searchsorted(db.edge_keys.numpy(), (r * E + t) * E + h)
        assert db.edge_ids.numpy()[j] == graph.relation2ht2index[r][graph.encode_ht(h, t)]


def test_device_eval_batches_tables():
    """The filter lists behind data.DeviceEvalBatches (hr2oo for valid, hr2ooo
    for test; reference src/data.py:250-255, 287-291) as an ascending-key CSR."""
    import numpy as np
    import torch
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import DeviceEvalBatches, KnowledgeGraph, TestDataset, ValidDataset
    graph = KnowledgeGraph(datasets.materialize("umls"))
    for ds, lists in ((ValidDataset(graph, 32), graph.hr2oo), (TestDataset(graph, 32), graph.hr2ooo)):
        db = DeviceEvalBatches(ds, torch.device("cpu"))
        keys, offs, vals = db.lists.keys.numpy(), db.lists.offs.numpy(), db.lists.vals.numpy()
        assert (np.diff(keys) > 0).all() and len(keys) == len(lists)
        for k, v in list(lists.items())[::13]:
            i = np.searchsorted(keys, k)
            assert keys[i] == k and list(vals[offs[i]:offs[i + 1]]) == v


def test_host_resources_keyed_by_stream_device(tmp_path):
    """The forward's per-device host resources (pinned header, side streams)
    are keyed by the device of the call's stream, not the thread's current
    device, and the current device is restored (csrc/hostside.h, as used by
    ground.hip's entry points) — with a mock device API, no GPU."""
    import subprocess
    exe = str(tmp_path / "hostside_keying")
    src = os.path.join(REPO, "tests", "native", "hostside_keying.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(REPO, "rnnlogic_amd", "csrc"), src,
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr
