"""Pin the C path-counting oracle (oracle/ground_oracle.c) to the reference:
  * the golden per-rule COO counts produced by the reference's Python grounding
  * the reference's own C++ rule_destination (oracle/_ref/libref_miner.so),
    compiled from /root/reference/miner (skipped where that build is absent).
Exact integer equality throughout."""
import os

import numpy as np
import pytest

from conftest import ALL_CASES
from oracle import ground_c
from oracle import reference_np as ref

_cache = {}


def setup(fx):
    p = fx.dataset_path()
    if p not in _cache:
        g = ref.Graph(p)
        cg = ground_c.CGraph(g.entity_size, g.relation_size, g.train_facts)
        rules = ref.Rules(fx.rule_path(), g.relation_size)
        _cache[p] = (g, ground_c.Oracle(cg, rules.rules, g.relation_size), rules)
    return _cache[p]


def coo_to_candidates(coo, B):
    out = []
    mix = {}
    for b in range(B):
        sel = coo[coo[:, 1] == b]
        acc = {}
        for rid, _, e, c in sel.tolist():
            if rid not in mix:
                mix[rid] = ground_c.mix64(rid)
            s, f = acc.get(e, (0, 0))
            acc[e] = (s + c, (f + c * mix[rid]) & 0xFFFFFFFFFFFFFFFF)
        keys = sorted(acc)
        out.append((np.asarray(keys, np.int64), np.asarray([acc[k][0] for k in keys], np.int64),
                    np.asarray([acc[k][1] for k in keys], np.uint64)))
    return out


@pytest.mark.parametrize("case", ALL_CASES)
def test_c_oracle_matches_golden_counts(case, fixtures):
    fx = fixtures(case)
    g, orc, _ = setup(fx)
    for k in range(min(fx.ncalls, 8)):
        c = fx.call(k)
        q = int(c["r"][0])
        want = coo_to_candidates(c["coo"].astype(np.int64), len(c["h"]))
        for b in range(len(c["h"])):
            rs = rd = -1
            if c["etr"] is not None:
                heads, tails = g.adj[q]
                rs, rd = int(heads[c["etr"][b]]), int(tails[c["etr"][b]])
            t, s, f = orc.candidates(int(c["h"][b]), q, rs, rd)
            np.testing.assert_array_equal(t, want[b][0])
            np.testing.assert_array_equal(s, want[b][1])
            np.testing.assert_array_equal(f, want[b][2])


@pytest.mark.skipif(not os.path.isdir("/root/reference/miner") and not os.path.exists(ground_c.REF_LIB),
                    reason="reference miner build unavailable")
@pytest.mark.parametrize("case", ["umls_lstm_sum_bias", "kinship_lstm_sum_none", "fb_lstm_sum_bias"])
def test_c_oracle_matches_reference_miner(case, fixtures):
    fx = fixtures(case)
    g, orc, rules = setup(fx)
    miner = ground_c.RefMiner(fx.dataset_path())
    rng = np.random.RandomState(3)
    facts = np.asarray(g.train_facts)
    qs = facts[rng.choice(len(facts), 12, replace=False)]
    try:
        for h, r, t in qs.tolist():
            acc = {}
            for rid, (hd, body) in rules.relation2rules[r]:
                d, cnt = miner.rule_destination(h, body, (h, r, t))
                m = ground_c.mix64(rid)
                for e, c in zip(d.tolist(), cnt.tolist()):
                    s, f = acc.get(e, (0, 0))
                    acc[e] = (s + c, (f + c * m) & 0xFFFFFFFFFFFFFFFF)
            tt, ss, ff = orc.candidates(h, r, h, t)
            keys = sorted(acc)
            np.testing.assert_array_equal(tt, keys)
            np.testing.assert_array_equal(ss, [acc[x][0] for x in keys])
            np.testing.assert_array_equal(ff, np.asarray([acc[x][1] for x in keys], np.uint64))
    finally:
        miner.close()


def test_c_oracle_digest_consistency(fixtures):
    """Batch digests equal digests recomputed from per-query candidate lists."""
    fx = fixtures("kinship_lstm_sum_none")
    g, orc, _ = setup(fx)
    facts = np.asarray(g.test_facts[:64])
    d, n = orc.digests(facts[:, 0], facts[:, 1], threads=4)
    for i, (h, r, t) in enumerate(facts.tolist()):
        tt, ss, ff = orc.candidates(h, r)
        acc = 0
        for a, b, c in zip(tt.tolist(), ss.tolist(), ff.tolist()):
            acc = (acc + ground_c.mix64(a ^ ground_c.mix64(b ^ ground_c.mix64(c)))) & 0xFFFFFFFFFFFFFFFF
        assert int(d[i]) == acc and n[i] == len(tt)


@pytest.mark.parametrize("name", ["FB15k-237", "kinship", "wn18rr"])
def test_bench_work_counts_fixture(name):
    """tests/golden/<name>_work.json (bench.py's algorithmic-bytes inputs)
    describes the bench rows, and its first 2000 queries re-derive from the C
    oracle."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("make_work_counts", os.path.join(root, "tools", "make_work_counts.py"))
    mwc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mwc)
    with open(mwc.out_path(name)) as f:
        w = json.load(f)
    graph, model, rows = mwc.workload(name)
    assert w["queries"] == len(rows) and w["rules"] == model.num_rules
    assert w["rows_sha256"] == mwc.rows_digest(rows)
    pre = w["prefix"]
    work, ncand = mwc.work_counts(graph, model, rows[:pre["queries"]], threads=os.cpu_count() or 1)
    assert [int(x) for x in work.sum(0)] == [pre["F"], pre["T"], pre["P"]]
    assert int(ncand.sum()) == pre["C"]
