"""PredictorPlus with hidden_dim != 16 (the reference accepts any size,
src/predictors.py:122): the fused scoring kernels are specialised for 16, so
other sizes run the HIP grounding and the aggregation / MLP as torch ops on
the grounding COO (PredictorPlus.forward_coo) — on the GPU, no CPU path.
Scores and masks against the numpy restatement of the reference
(oracle/reference_np.py) on UMLS test batches, eval and train mode (edge
removal), and one training step's loss is finite with gradients on every
used parameter."""
import numpy as np
import pytest
import torch

from oracle import reference_np as ref

pytestmark = pytest.mark.gpu

CASES = [(8, "emb", "sum", "bias"), (32, "lstm", "pna", "none"), (24, "lstm", "sum", "bias")]


@pytest.mark.parametrize("H,typ,agg,feature", CASES)
def test_hidden_dim_matches_oracle(H, typ, agg, feature):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, TrainDataset
    from rnnlogic_amd.predictors import PredictorPlus
    dev = torch.device("cuda:0")
    path = datasets.materialize("umls")
    torch.manual_seed(0)
    graph = KnowledgeGraph(path)
    model = PredictorPlus(graph, type=typ, num_layers=2, hidden_dim=H, entity_feature=feature, aggregator=agg)
    model.set_rules(datasets.rule_file("umls"))
    if feature == "bias":
        with torch.no_grad():
            model.bias.normal_()
    model = model.to(dev).eval()
    assert not model.fused
    g = ref.Graph(path)
    rules = ref.Rules(datasets.rule_file("umls"), g.relation_size)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    cfg = dict(type=typ, aggregator=agg, entity_feature=feature, num_layers=2)
    test = np.asarray(graph.test_facts, dtype=np.int64)
    worst = 0.0
    for rel in np.unique(test[:, 1])[:6]:
        rows = test[test[:, 1] == rel][:32]
        h = torch.from_numpy(rows[:, 0]).to(dev)
        r = torch.from_numpy(rows[:, 1]).to(dev)
        with torch.no_grad():
            score, mask = model(h, r, None)
        want, wmask = ref.predictorplus_forward(sd, cfg, g, rules, rows[:, 0], rows[:, 1], None)
        got = score.cpu().numpy()
        assert np.array_equal(mask.cpu().numpy(), wmask)
        fin = np.isfinite(want)
        np.testing.assert_array_equal(np.isfinite(got), fin)
        if fin.any():
            worst = max(worst, float(np.abs(got[fin] - want[fin]).max()))
    assert worst <= 1e-4, worst
    # train mode: edge removal, autograd through the same COO path
    model.train()
    ts = TrainDataset(graph, 32)
    all_h, all_r, all_t, target, etr = ts[0]
    logits, mask = model(all_h.to(dev), all_r.to(dev), etr.to(dev))
    if mask.sum().item():
        loss = -(torch.log_softmax(logits, 1)[mask] * target.to(dev)[mask]).sum()
        loss.backward()
        assert torch.isfinite(loss)
        assert model.score_model.layers[0].weight.grad is not None
    print("H=%d %s/%s/%s: max |score - oracle| %.3g" % (H, typ, agg, feature, worst))
