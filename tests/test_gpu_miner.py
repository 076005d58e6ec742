"""GPU rule mining (rnnl_rule_search, rnnlogic_amd/miner.py) against the
reference miner's own rule pools (tests/golden/rules_*.npz, made by
tools/make_golden_rules.py from RuleMiner::search compiled from
/root/reference/miner).  Exact set and order equality."""
import numpy as np
import pytest
import torch

from conftest import RULE_CASES, golden_rules

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("case", RULE_CASES)
def test_rule_search_matches_reference_miner(case, dev):
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.miner import RuleMiner
    _, data, L = case.split("_")
    miner = RuleMiner(KnowledgeGraph(datasets.materialize(data)), dev)
    got = miner.search(int(L[1:]))
    want = golden_rules(case)
    assert len(got) == len(want)
    assert got == want


def test_rule_search_small_table_retries(dev):
    """A table too small for the pool is reported and the search retried."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.miner import RuleMiner
    miner = RuleMiner(KnowledgeGraph(datasets.materialize("umls")), dev)
    miner.table_bits = 10
    assert miner.search(3) == golden_rules("rules_umls_L3")
    assert miner.table_bits > 10


def test_rule_search_save_format(dev, tmp_path):
    """RuleMiner.save writes RuleMiner::save's format, readable by set_rules."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.miner import RuleMiner
    miner = RuleMiner(KnowledgeGraph(datasets.materialize("kinship")), dev)
    rules = miner.search(2)
    p = tmp_path / "rules.txt"
    assert miner.save(str(p)) == len(rules)
    lines = p.read_text().splitlines()
    for (hd, body), line in zip(rules, lines):
        tok = line.split()
        assert int(tok[0]) == len(body) and int(tok[1]) == hd
        assert tuple(int(x) for x in tok[2:2 + len(body)]) == body
        assert np.allclose([float(x) for x in tok[2 + len(body):]], 0.0)
