"""Run-to-run determinism of training (deterministic kernels,
ordered reductions).

The same seeded model trained for 20 batches twice through
TrainerPredictor.train (device batches, the grounding lookahead, the fused
HIP forward and backward) must end with bitwise-equal parameters.  The
backward's reductions that used to be atomic sums in arbitrary order are
now order-independent: the RotatE d(h o r) partials are summed per entity
block in block order (rotate.hip head_grad_kernel), the SUM rule part's
per-node gradients and the EM Predictor's are int64 fixed-point sums at
one scale per launch (backward.hip node_accum_kernel, predictor.hip
predictor_backward_kernel), and relation_emb's gradient of a one-relation
batch is W0[:, 16:]^T dL/db0 in a fixed order (rel_grad_kernel).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

N_BATCHES = 20


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _bits(t):
    t = t.detach().cpu().contiguous()
    return t.view(torch.int32) if t.dtype == torch.float32 else t


def _train(dev, data, kind, kw, dim):
    import contextlib
    import io

    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.predictors import Predictor, PredictorPlus
    from rnnlogic_amd.trainer import TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    set_seed(1)
    with contextlib.redirect_stdout(io.StringIO()):
        graph = KnowledgeGraph(datasets.materialize(data, with_rotate=dim is not None))
        train_set = TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        TestDataset(graph, 32)
        if kind == "plus":
            model = PredictorPlus(graph, num_layers=3, hidden_dim=16,
                                  embedding_path=datasets.rotate_path(data) if dim else None, **kw)
        else:
            model = Predictor(graph, **kw)
        model.set_rules(datasets.rule_file(data))
    if kind != "plus":
        with torch.no_grad():
            model.rule_weights.normal_(0.0, 0.1)
    optim = torch.optim.Adam(model.parameters(), lr=5e-3, weight_decay=0)
    solver = TrainerPredictor(model, train_set, None, None, optim, gpus=[dev.index or 0])
    solver.train(batch_per_epoch=N_BATCHES, smoothing=0.2, print_every=10 ** 9)
    torch.cuda.synchronize(dev)
    return {k: _bits(v) for k, v in solver.model.state_dict().items()}


CASES = {
    # the headline model (config 4): LSTM encoder backward, fused SUM
    # backward, RotatE D = 1000 parameter gradients
    "fb_lstm_sum_rotate": ("FB15k-237", "plus", dict(type="lstm", entity_feature="RotatE", aggregator="sum"), 1000),
    # config 5's final PredictorPlus
    "fb_emb_sum_bias": ("FB15k-237", "plus", dict(type="emb", entity_feature="bias", aggregator="sum"), None),
    # config 5's EM rule-weight Predictor
    "fb_em_predictor": ("FB15k-237", "pred", dict(entity_feature="bias"), None),
    "kinship_lstm_sum_none": ("kinship", "plus", dict(type="lstm", entity_feature="none", aggregator="sum"), None),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_training_is_bitwise_repeatable(case, dev):
    data, kind, kw, dim = CASES[case]
    a = _train(dev, data, kind, kw, dim)
    b = _train(dev, data, kind, kw, dim)
    assert a.keys() == b.keys()
    differ = [k for k in a if not torch.equal(a[k], b[k])]
    assert not differ, "%s: parameters differ between two identical runs: %s" % (case, differ)
