"""Golden rule pools from the REFERENCE miner (RuleMiner::search, compiled from
/root/reference/miner into oracle/_ref): tests/golden/rules_<data>_L<n>.npz
with `flat` = (head, len, body...) in the reference's order.

Usage: python tools/make_golden_rules.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import ground_c  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402

for data in ("umls", "kinship"):
    for L in (2, 3):
        m = ground_c.RefMiner(datasets.materialize(data))
        rules, sec = m.rule_search(L, threads=8)
        m.close()
        flat = []
        for hd, body in rules:
            flat += [hd, len(body)] + list(body)
        out = os.path.join(REPO, "tests", "golden", "rules_%s_L%d.npz" % (data, L))
        np.savez_compressed(out, flat=np.asarray(flat, dtype=np.int16 if max(flat) < 32767 else np.int32),
                            seconds=sec)
        print(out, len(rules), "rules, reference search %.2f s (8 threads)" % sec)
