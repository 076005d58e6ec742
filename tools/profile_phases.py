"""Per-phase cycle breakdown of the fused forward kernel (diagnostic; GPU box).

Runs the bench workload's grounding kernel once with rnnl_debug_profile
counters and prints cycles per query for each phase, plus event timings of
the three launches.  Usage: python tools/profile_phases.py [--feature bias]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402


def main():
    import faulthandler
    faulthandler.dump_traceback_later(int(os.environ.get("HANG_DUMP_S", "60")), exit=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--feature", default="bias")
    ap.add_argument("--rows", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    graph, test_set, model, rows = bench.build_workload(args.feature)
    if args.rows:
        rows = rows[:args.rows]
    model = model.to(dev).eval()
    h = torch.from_numpy(rows[:, 0]).to(dev)
    r = torch.from_numpy(rows[:, 1]).to(dev)
    with torch.no_grad():
        model.forward_rows(h, r, None)
        prof = torch.zeros(13, dtype=torch.int64, device=dev)
        _native.call("rnnl_debug_profile", prof.data_ptr())
        ev = {}
        model.forward_rows(h, r, None, events=ev)
        torch.cuda.synchronize()
        _native.call("rnnl_debug_profile", None)
    p = prof.cpu().tolist()
    nq = max(p[3], 1)
    print("queries %d  contributions/q %.1f  candidates/q %.1f" % (p[3], p[4] / nq, p[5] / nq))
    for name, v in zip(["prologue", "grounding(A)", "candidates(B)"], p[:3]):
        print("  %-14s %10.0f cycles/query" % (name, v / nq))
    for name, v in zip(["B mark+slots", "B count+records", "B scatter", "A node+scan", "A item+scan",
                        "A edges", "A compaction"], p[6:13]):
        print("  %-14s %10.0f cycles/query" % (name, v / nq))
    print("events ms: nodes %.3f base %.3f ground %.3f" % (ev["start"].elapsed_time(ev["base"]),
          ev["base"].elapsed_time(ev["ground"]), ev["ground"].elapsed_time(ev["end"])))


if __name__ == "__main__":
    main()
