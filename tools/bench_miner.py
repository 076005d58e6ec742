"""GPU rule search (rnnlogic_amd.miner.RuleMiner) timings: rules found and
seconds per (dataset, max_length); the reference miner's CPU time for the
same pools where the golden fixtures recorded it (8 threads, this build
container).  Usage: python tools/bench_miner.py [data:L ...]"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph  # noqa: E402
from rnnlogic_amd.miner import RuleMiner  # noqa: E402


def main():
    cases = sys.argv[1:] or ["umls:3", "kinship:3", "wn18rr:3", "FB15k-237:2", "FB15k-237:3"]
    dev = torch.device("cuda:0")
    for c in cases:
        data, L = c.split(":")
        with contextlib.redirect_stdout(io.StringIO()):
            g = KnowledgeGraph(datasets.materialize(data))
        m = RuleMiner(g, dev)
        print("mining %s L=%s ..." % (data, L), flush=True)
        m.search(int(L))  # warm-up (and table sizing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        keys = m.search_keys(int(L))
        torch.cuda.synchronize()
        sec = time.perf_counter() - t0
        ref = os.path.join(REPO, "tests", "golden", "rules_%s_L%s.npz" % (data, L))
        ref_s = float(np.load(ref)["seconds"]) if os.path.exists(ref) else None
        print(json.dumps({"data": data, "max_length": int(L), "triples": len(g.train_facts), "rules": int(len(keys)),
                          "gpu_s": round(sec, 4), "reference_cpu_s_8_threads": ref_s}), flush=True)


if __name__ == "__main__":
    main()
