"""HIP path parity (runs on the MI355X box).

Every forward goes through the C-ABI library (rnnlogic_amd/_build/
librnnlogic_hip.so).  Checks, against the reference's own outputs
(tests/golden) and the C oracle (oracle/ground_oracle.c):
  * entity scores within 1e-4 (fp32, abs) and identical masks;
  * exact integer parity of the per-rule path counts, through the
    order-independent digest of (candidate, sum of counts, rule fingerprint)
    — on the fixture batches and on the FULL synthetic FB15k-237 test split;
  * candidate counts per query;
  * RotatE known-answer MRRs of the shipped embeddings (train.log values).
"""
import numpy as np
import pytest
import torch

from conftest import ALL_CASES, Fixture
from oracle import ground_c
from oracle import reference_np as ref

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north_star: entity scores within 1e-4 fp32

_graphs, _oracles = {}, {}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def graph_for(path):
    from rnnlogic_amd.data import KnowledgeGraph
    if path not in _graphs:
        _graphs[path] = KnowledgeGraph(path)
    return _graphs[path]


def oracle_for(fx):
    p = fx.dataset_path()
    if p not in _oracles:
        g = ref.Graph(p)
        rules = ref.Rules(fx.rule_path(), g.relation_size)
        cg = ground_c.CGraph(g.entity_size, g.relation_size, g.train_facts)
        _oracles[p] = (g, ground_c.Oracle(cg, rules.rules, g.relation_size))
    return _oracles[p]


def build_model(fx, dev):
    from rnnlogic_amd.predictors import PredictorPlus
    graph = graph_for(fx.dataset_path())
    cfg = dict(fx.cfg["model"])
    model = PredictorPlus(graph, embedding_path=fx.rotate_path(), **cfg)
    model.set_rules(fx.rule_path())
    sd = {k: torch.from_numpy(v) for k, v in fx.sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all(k.startswith("RotatE.") for k in missing), (missing, unexpected)
    return model.to(dev).eval()


@pytest.mark.parametrize("case", ALL_CASES)
def test_forward_matches_reference(case, dev):
    fx = Fixture(case)
    model = build_model(fx, dev)
    worst = 0.0
    for k in range(fx.ncalls):
        c = fx.call(k)
        h = torch.from_numpy(c["h"]).to(dev)
        r = torch.from_numpy(c["r"]).to(dev)
        etr = torch.from_numpy(c["etr"]).to(dev) if c["etr"] is not None else None
        with torch.no_grad():
            score, mask = model(h, r, etr)
        score = score.cpu().numpy()
        np.testing.assert_array_equal(mask.cpu().numpy(), c["mask"], err_msg="%s call %d mask" % (case, k))
        want = c["score"]
        fin = np.isfinite(want)
        np.testing.assert_array_equal(np.isfinite(score), fin)
        np.testing.assert_array_equal(score[~fin], want[~fin])
        if fin.any():
            err = float(np.abs(score[fin] - want[fin]).max())
            worst = max(worst, err)
            assert err <= TOL, "%s call %d: max |score - reference| = %g" % (case, k, err)
    print("%s: %d calls, max abs err %.3g" % (case, fx.ncalls, worst))


@pytest.mark.parametrize("case", ALL_CASES)
def test_path_count_digests(case, dev):
    """Exact integer parity of the grounding for every fixture batch."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    g, orc = oracle_for(fx)
    for k in range(fx.ncalls):
        c = fx.call(k)
        rs = rd = None
        if c["etr"] is not None:
            q = int(c["r"][0])
            heads, tails = g.adj[q]
            rs, rd = heads[c["etr"]], tails[c["etr"]]
        want_d, want_n = orc.digests(c["h"], c["r"], rs, rd, threads=4)
        h = torch.from_numpy(c["h"]).to(dev)
        r = torch.from_numpy(c["r"]).to(dev)
        etr = torch.from_numpy(c["etr"]).to(dev) if c["etr"] is not None else None
        dig = torch.zeros(len(h), dtype=torch.int64, device=dev)
        with torch.no_grad():
            _, _, ncand = model.forward_rows(h, r, etr, return_ncand=True, digest=dig)
        np.testing.assert_array_equal(ncand.cpu().numpy(), want_n)
        np.testing.assert_array_equal(dig.cpu().numpy().view(np.uint64), want_d)


@pytest.mark.parametrize("case", ["fb_lstm_sum_bias", "wn_emb_pna_bias", "kinship_lstm_sum_none"])
def test_full_test_split_digests(case, dev):
    """Size-independent property at full size: every test query of the
    synthetic FB15k-237 graph (40,932, rules L <= 3, sum), of WN18RR
    (6,268, rules L <= 5, PNA: its two phase-B sweeps) and of kinship (5,343,
    config 2's exact model: mined L <= 3 rules, no entity feature) grounds to
    exactly the oracle's path counts (digest + candidate count), 8,192 rows
    per launch."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    g, orc = oracle_for(fx)
    test = np.asarray(g.test_facts, dtype=np.int64)
    want_d, want_n = orc.digests(test[:, 0], test[:, 1])
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    got_d, got_n = [], []
    for s in range(0, len(test), 8192):
        dig = torch.zeros(min(8192, len(test) - s), dtype=torch.int64, device=dev)
        with torch.no_grad():
            _, _, n = model.forward_rows(h[s:s + 8192], r[s:s + 8192], None, return_ncand=True, digest=dig)
        got_d.append(dig.cpu().numpy().view(np.uint64))
        got_n.append(n.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(got_n), want_n)
    np.testing.assert_array_equal(np.concatenate(got_d), want_d)


@pytest.mark.parametrize("case", ["umls_emb_pna_rotate", "fb_lstm_sum_rotate"])
def test_stream_overlap_is_bit_identical(case, dev):
    """RotatE forwards overlap the grounding and the scoring pass (side
    stream, atomic adds into zeroed rows) with RotatE: bit-identical scores,
    candidate counts and path-count digests to the one-stream launch, on all
    test rows of the graph at once (mixed relations, many reference
    batches)."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    test = np.asarray(graph_for(fx.dataset_path()).test_facts, dtype=np.int64)[:6000]
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    outs = []
    for overlap in (False, True):
        model.overlap = overlap
        dig = torch.zeros(len(h), dtype=torch.int64, device=dev)
        with torch.no_grad():
            score, mask, n = model.forward_rows(h, r, None, return_ncand=True, digest=dig)
        torch.cuda.synchronize()
        outs.append((score.cpu().numpy(), mask.cpu().numpy(), n.cpu().numpy(), dig.cpu().numpy()))
    model.overlap = True
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)
    g, orc = oracle_for(fx)
    want_d, want_n = orc.digests(test[:, 0], test[:, 1])
    np.testing.assert_array_equal(outs[0][2], want_n)
    np.testing.assert_array_equal(outs[0][3].view(np.uint64), want_d)


@pytest.mark.parametrize("case", ["fb_lstm_sum_bias", "kinship_lstm_sum_none", "wn_emb_pna_bias"])
def test_ground_early_is_bit_identical(case, dev):
    """Without RotatE the grounding runs on a side stream beside the rule
    encoder (PredictorPlus.ground_early, the split ground / score entries):
    scores, masks and candidate counts equal the one-call launch's."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    test = np.asarray(graph_for(fx.dataset_path()).test_facts, dtype=np.int64)[:6000]
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    outs = []
    for early in (False, True):
        model.ground_early = early
        model.invalidate_cache()
        with torch.no_grad():
            score, mask, n = model.forward_rows(h, r, None, return_ncand=True)
        torch.cuda.synchronize()
        outs.append((score.cpu().numpy(), mask.cpu().numpy(), n.cpu().numpy()))
    model.ground_early = True
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("case", ["fb_lstm_sum_bias", "fb_lstm_sum_rotate", "kinship_lstm_sum_none",
                                  "umls_lstm_sum_bias"])
def test_pair_memo_is_bit_identical(case, dev):
    """The SUM pair memo (score_model outputs keyed by a candidate's one or
    two bucket entries, ground.hip pair_key) reuses outputs of equal features:
    scores, masks and candidate counts equal the launch without it, one stream
    and overlapped, over many relation batches of the test split."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    test = np.asarray(graph_for(fx.dataset_path()).test_facts, dtype=np.int64)[:8000]
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    from rnnlogic_amd import _native
    outs = []
    try:
        for on, overlap in ((0, False), (1, False), (1, True)):
            _native.call("rnnl_debug_pair_memo", on)
            model.overlap = overlap
            with torch.no_grad():
                out = model.forward_rows(h, r, None, return_ncand=True)
            torch.cuda.synchronize()
            outs.append([x.cpu().numpy() for x in out])
    finally:
        _native.call("rnnl_debug_pair_memo", 1)
    model.overlap = True
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("case", ["fb_lstm_sum_bias", "umls_emb_pna_rotate", "kinship_lstm_sum_none"])
def test_dedupe_is_bit_identical(case, dev):
    """forward_rows(dedupe=True) computes each distinct (h, r) once: same
    scores, masks and candidate counts as the row-by-row forward."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    test = np.asarray(graph_for(fx.dataset_path()).test_facts, dtype=np.int64)[:4000]
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    with torch.no_grad():
        a = model.forward_rows(h, r, None, return_ncand=True)
        b = model.forward_rows(h, r, None, return_ncand=True, dedupe=True)
    assert len(torch.unique(r * 100000 + h)) < len(h)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())


@pytest.mark.parametrize("data,dim,mrr", [("umls", 200, 0.659847), ("umls", 50, 0.344034),
                                          ("kinship", 1000, 0.637454)])
def test_rotate_known_answer_mrr(data, dim, mrr, dev):
    """RotatE HIP scorer reproduces the shipped train.log test MRR (KAT)."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.embedding import RotatE
    g = ref.Graph(datasets.materialize(data))
    rot = RotatE(datasets.rotate_path(data, dim)).to(dev)
    R = g.relation_size
    test = np.asarray(g.test_facts)
    allt = set(g.train_facts) | set(g.valid_facts) | set(g.test_facts)
    rr = []
    for side in ("tail", "head"):
        hh = test[:, 0] if side == "tail" else test[:, 2]
        rel = test[:, 1] if side == "tail" else test[:, 1] + R
        tt = test[:, 2] if side == "tail" else test[:, 0]
        with torch.no_grad():
            s = rot(torch.from_numpy(hh).to(dev), torch.from_numpy(rel).to(dev)).cpu().numpy()
        for k in range(len(test)):
            row = s[k].copy()
            h0, r0, t0 = (int(x) for x in test[k])
            for e in range(g.entity_size):
                trip = (h0, r0, e) if side == "tail" else (e, r0, t0)
                if e != tt[k] and trip in allt:
                    row[e] = -np.inf
            rr.append(1.0 / (1 + int((row > row[tt[k]]).sum())))
    assert abs(float(np.mean(rr)) - mrr) < 5e-7, (float(np.mean(rr)), mrr)


def _rotate_f64(eemb, remb, gamma, h, r):
    """float64 restatement of embedding.py:45-70 (fp32 phase divisor)."""
    D = eemb.shape[1] // 2
    div = np.float32((gamma + 2.0) / D / np.pi)
    ph = (remb[r] / div).astype(np.float64)
    e = eemb.astype(np.float64)
    hh = e[h]
    re = hh[:, :D] * np.cos(ph) - hh[:, D:] * np.sin(ph)
    im = hh[:, :D] * np.sin(ph) + hh[:, D:] * np.cos(ph)
    out = np.empty((len(h), e.shape[0]))
    for i in range(len(h)):
        out[i] = gamma - np.sqrt((re[i][None] - e[:, :D]) ** 2 + (im[i][None] - e[:, D:]) ** 2).sum(1)
    return out


@pytest.mark.parametrize("source", ["kinship1000", "umls200", "scale0.5", "near-match", "identity-self"])
@pytest.mark.parametrize("mode", ["mfma", "direct"])
def test_rotate_scores_vs_float64(source, mode, dev):
    """RotatE kernels against a float64 evaluation of embedding.py:45-70: the
    shipped trained tables, a large-magnitude table, and queries whose h o r
    nearly equals some entity (the cancellation regime of the expanded MFMA
    form).  The default DIRECT kernel is within 1e-4 (fp32, abs) everywhere;
    the opt-in MFMA kernel is within 1e-4 on the real and random tables and
    within its documented bound on the adversarial near-match rows.  Also
    checks accumulate=1 and ragged shapes (E, B not multiples of the tiles)."""
    from rnnlogic_amd import _native, datasets
    from rnnlogic_amd.embedding import RotatE
    name, dim = ("kinship", 1000) if source == "kinship1000" else ("umls", 200)
    rot = RotatE(datasets.rotate_path(name, dim))
    rng = np.random.default_rng(7)
    R2 = rot.remb.shape[0]
    h = rng.integers(0, rot.num_entities, 37)
    r = rng.integers(0, R2, 37)
    if source == "scale0.5":
        with torch.no_grad():
            rot.eemb.copy_(torch.from_numpy(rng.uniform(-0.5, 0.5, rot.eemb.shape).astype(np.float32)))
    if source == "near-match":
        # make entity t_i = h_i o r_i (+ tiny noise) for the first rows
        e = rot.eemb.detach().numpy().astype(np.float64)
        D = rot.emb_dim
        div = np.float32((rot.gamma + 2.0) / D / np.pi)
        ph = rot.remb.detach().numpy()[r] / div
        for i in range(8):
            hr_re = e[h[i], :D] * np.cos(ph[i]) - e[h[i], D:] * np.sin(ph[i])
            hr_im = e[h[i], :D] * np.sin(ph[i]) + e[h[i], D:] * np.cos(ph[i])
            t = (h[i] + 1 + i) % rot.num_entities
            e[t, :D] = hr_re + rng.normal(0, 1e-6, D)
            e[t, D:] = hr_im + rng.normal(0, 1e-6, D)
        with torch.no_grad():
            rot.eemb.copy_(torch.from_numpy(e.astype(np.float32)))
    if source == "identity-self":
        # a relation with zero phases (a symmetric relation's learned 0-phase
        # dims, taken to the limit): the candidate e = h sits at distance 0
        with torch.no_grad():
            rot.remb[r[:8]] = 0.0
    want = _rotate_f64(rot.eemb.detach().numpy(), rot.remb.detach().numpy(), rot.gamma, h, r)
    rot = rot.to(dev)
    rot.mode = _native.ROTATE_MFMA if mode == "mfma" else _native.ROTATE_DIRECT
    hh = torch.from_numpy(h).to(dev)
    rr = torch.from_numpy(r).to(dev)
    with torch.no_grad():
        got = rot(hh, rr).cpu().numpy()
        base = torch.full((len(h), rot.num_entities), 0.25, device=dev)
        rot.score_into(hh, rr, base, accumulate=True)
    err = float(np.abs(got - want).max())
    np.testing.assert_allclose(base.cpu().numpy(), got + 0.25, rtol=0, atol=2e-6)
    if source == "identity-self":
        assert np.all(got[np.arange(8), h[:8]] == np.float32(rot.gamma)) or mode == "mfma"
    if mode == "mfma" and source in ("near-match", "identity-self"):
        # The expanded form's documented limit (DESIGN.md "RotatE numerics"):
        # |err| <= sum_d sqrt(c 2^-24 (|hr_d|^2 + |t_d|^2)), c = 8 — here the
        # default DIRECT kernel is the one that meets TOL.
        e = rot.eemb.detach().cpu().numpy().astype(np.float64)
        D = rot.emb_dim
        nrm_t = e[:, :D] ** 2 + e[:, D:] ** 2
        bound = np.sqrt(8 * 2.0 ** -24 * (nrm_t[h[:8]] * 2)).sum(1).max()  # |hr| = |h| (unit rotation)
        assert err <= bound, (err, bound)
        return
    assert err <= TOL, "%s/%s: max |score - f64| = %g" % (source, mode, err)


@pytest.mark.parametrize("data", ["umls", "kinship", "FB15k-237", "wn18rr"])
def test_lstm_encoder_matches_torch(data, dev):
    """rnnl_lstm_encode == PredictorPlus.encode_rules (torch LSTM) for every rule."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.predictors import PredictorPlus
    torch.manual_seed(3)
    graph = graph_for(datasets.materialize(data))
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16)
    model.set_rules(datasets.rule_file(data))
    model = model.to(dev).eval()
    with torch.no_grad():
        want = model.encode_rules(model.rule_features.to(dev))
        got = model._encode_rules_hip(dev)
        model.encoder_trie = False
        per_rule = model._encode_rules_hip(dev)
    err = float((got - want).abs().max())
    assert err <= 2e-6, err
    # the trie form (one step per prefix) is bitwise the per-rule encoder
    assert torch.equal(got, per_rule)
    # the SUM node records formed inside the trie encoder's launches
    # (rnnl_lstm_encode_trie_sum) are bitwise rnnl_node_weights' table of its rows
    import ctypes
    from rnnlogic_amd import _native
    model.encoder_trie = True
    assert model.aggregator == "sum"
    nr = model.native_rules(dev)
    add_w = model.rule_to_entity.add_model.layers[0].weight.detach().float().contiguous()
    nbytes = ctypes.c_size_t()
    _native.call("rnnl_node_weights_size", nr.ptr, _native.AGG_SUM, ctypes.byref(nbytes))
    fused = torch.full((nbytes.value,), 0xAB, dtype=torch.uint8, device=dev)
    with torch.no_grad():
        emb = model._encode_rules_hip(dev, add_w, fused)
    assert torch.equal(emb, got)
    sep = torch.full_like(fused, 0xCD)
    _native.call("rnnl_node_weights", nr.ptr, got.data_ptr(), got.stride(0), _native.AGG_SUM, add_w.data_ptr(),
                 sep.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    n_rec = nbytes.value - 64  # the records; then the trailer's 32 written bytes
    assert torch.equal(fused[:n_rec + 32], sep[:n_rec + 32])
    assert torch.equal(model.node_weights(dev)[:n_rec + 32], sep[:n_rec + 32])


@pytest.mark.parametrize("data", ["FB15k-237", "umls"])
def test_rotate_split_form_is_bitwise(data, dev):
    """A launch with few rows (one 32-row reference batch) runs RotatE in the
    split-dimension form (rotate_split_kernel + rotate_combine_kernel); its
    scores equal the one-pass direct kernel's bitwise for the same rows —
    including ragged row counts and the accumulate mode."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.embedding import RotatE
    path = datasets.rotate_path(data) if data == "FB15k-237" else datasets.rotate_path(data, 200)
    rot = RotatE(path).to(dev)
    E = rot.num_entities
    g = torch.Generator().manual_seed(3)
    n_big = 4096 if data == "FB15k-237" else 40000  # enough rows for the one-pass grid
    h = torch.randint(0, E, (n_big,), generator=g).to(dev)
    r = torch.randint(0, rot.remb.shape[0], (n_big,), generator=g).to(dev)
    with torch.no_grad():
        big = rot(h, r)
        for n in (32, 7, 45):
            small = rot(h[:n], r[:n])
            assert torch.equal(small, big[:n]), (n, float((small - big[:n]).abs().max()))
        base = torch.randn(5, E, device=dev)
        acc = rot.score_into(h[:5], r[:5], base.clone(), accumulate=True)
        assert torch.equal(acc, base + big[:5])
        # the one-pass grid in several launches (rnnl_rotate_score_pieces, the
        # PNA overlap's yield point): the same blocks, bitwise the same scores
        for pieces, share in ((2, 0.5), (2, 0.37), (3, 0.0), (5, 0.1)):
            out = torch.full_like(big, float("nan"))
            rot.score_into(h, r, out, pieces=pieces, first_share=share)
            assert torch.equal(out, big), (pieces, share)
            zero = torch.zeros_like(big)
            rot.score_into(h, r, zero, accumulate=2, pieces=pieces, first_share=share)
            assert torch.equal(zero, big), ("atomic", pieces, share)


@pytest.mark.parametrize("data", ["umls", "FB15k-237"])
def test_lstm_train_path_matches_torch(data, dev):
    """_LstmRules (rnnl_lstm_train_forward / _backward) == torch's LSTM under
    autograd (PredictorPlus.encode_rules) on the rules of single relations and
    of a mixed relation set: the outputs and every parameter gradient (the
    three layers' weights and biases and the vocab rows) for a random upstream
    gradient.  The vocab's padding row gets no gradient in either."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.predictors import PredictorPlus, _LstmRules  # noqa: F401
    torch.manual_seed(5)
    graph = graph_for(datasets.materialize(data))
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16)
    model.set_rules(datasets.rule_file(data))
    model = model.to(dev).train()
    counts = [len(x) for x in model.relation2rules]
    order = np.argsort(counts)[::-1]
    cases = [[int(order[0])], [int(order[len(order) // 3])], sorted(int(x) for x in order[1:4])]
    names = ["vocab_emb.weight"] + ["rnn.%s_l%d" % (n, k) for k in range(3)
                                    for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    params = dict(model.named_parameters())
    for rels in cases:
        if sum(counts[q] for q in rels) == 0:
            continue
        ridx = model._rule_ids(rels, dev)
        g = torch.randn(ridx.numel(), 16, generator=torch.Generator().manual_seed(len(rels))).to(dev)
        res = []
        for hip in (False, True):
            model.zero_grad()
            out = model._encode_rules_padded(ridx, dev, rels if hip else None)
            (out * g).sum().backward()
            res.append((out.detach().clone(), {n: params[n].grad.detach().clone() for n in names}))
        (o0, g0), (o1, g1) = res
        assert float((o0 - o1).abs().max()) <= 2e-6, rels
        for n in names:
            a, b = g0[n].cpu().numpy(), g1[n].cpu().numpy()
            scale = float(np.abs(a).max())
            np.testing.assert_allclose(b, a, atol=1e-5 * scale + 1e-6, rtol=1e-4, err_msg="%s %s" % (rels, n))
        assert float(g1["vocab_emb.weight"][model.padding_index].abs().max()) == 0.0
