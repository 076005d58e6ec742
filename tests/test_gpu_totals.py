"""rnnl_forward_status_totals: the grounding's candidate and bucket-entry
totals, read back with the status, size the COO export of the training path
(PredictorPlus.ground_coo) without further host syncs.  They must equal the
sum of n_cand and the sum of the exported bucket lengths, with and without
per-row edge removal (reference src/data.py:164-169), and ground_coo's COO
must match the oracle's per-row path counts (oracle/reference_np.py)."""
import numpy as np
import pytest
import torch

from oracle import reference_np as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("remove", [False, True])
def test_status_totals_size_the_coo(remove):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnlogic_amd import _native, datasets
    from rnnlogic_amd.data import KnowledgeGraph, TrainDataset
    from rnnlogic_amd.predictors import PredictorPlus
    dev = torch.device("cuda:0")
    path = datasets.materialize("umls")
    torch.manual_seed(0)
    graph = KnowledgeGraph(path)
    model = PredictorPlus(graph, type="emb", entity_feature="bias", aggregator="sum")
    model.set_rules(datasets.rule_file("umls"))
    model = model.to(dev)
    if remove:
        batch = TrainDataset(graph, 32)[0]
        h, r, etr = batch[0].to(dev), batch[1].to(dev), batch[4].to(dev)
    else:
        facts = graph.test_facts[:64]
        h = torch.tensor([f[0] for f in facts], device=dev)
        r = torch.tensor([f[1] for f in facts], device=dev)
        etr = None
    totals = np.zeros(2, dtype=np.int64)
    ws, scale, n_cand = model.ground(h, r, etr, totals)
    nq = h.numel()
    nc = n_cand.to(torch.int64)
    cand_off = torch.zeros(nq + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nc, 0, out=cand_off[1:])
    C = int(cand_off[-1])
    assert totals[0] == C > 0
    ent = torch.empty(C, dtype=torch.int32, device=dev)
    nent = torch.empty(C, dtype=torch.int32, device=dev)
    _native.call("rnnl_ground_export_candidates", ws.data_ptr(), nq, scale, n_cand.data_ptr(), cand_off.data_ptr(),
                 ent.data_ptr(), nent.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    assert totals[1] == int(nent.to(torch.int64).sum()) > 0
    # the COO sized by the totals carries the oracle's path counts
    row, ent_c, ce, node, count = model.ground_coo(h, r, etr)
    nr = model.native_rules(dev)
    g = ref.Graph(path)
    rules = ref.Rules(datasets.rule_file("umls"), g.relation_size)
    node_of_rule = nr.node_of_rule.cpu().numpy()
    got = {}
    for rw, e, n, c in zip(row[ce].tolist(), ent_c[ce].tolist(), node.tolist(), count.tolist()):
        got[(rw, e, n)] = got.get((rw, e, n), 0) + c
    hs, rs = h.cpu().numpy(), r.cpu().numpy()
    es = etr.cpu().numpy() if etr is not None else None
    rows_checked = range(0, nq, 7)
    want = {}
    for k in rows_checked:
        for i, (_, body) in rules.relation2rules[int(rs[k])]:
            cnt = ref.grounding(g, [int(hs[k])], int(rs[k]), body, None if es is None else [int(es[k])])[0]
            for e in np.nonzero(cnt)[0].tolist():
                want[(k, e, int(node_of_rule[i]))] = int(cnt[e])  # rules ending at one node count alike
    got_rows = {key: v for key, v in got.items() if key[0] in set(rows_checked)}
    assert got_rows == want
