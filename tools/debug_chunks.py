"""Diagnostic: run the bench workload's forward in row chunks, printing per
chunk wall time, overflow retries and candidate counts (GPU box)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    feature = sys.argv[1] if len(sys.argv) > 1 else "bias"
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda:0")
    graph, test_set, model, rows = bench.build_workload(feature)
    model = model.to(dev).eval()
    h = torch.from_numpy(rows[:, 0]).to(dev)
    r = torch.from_numpy(rows[:, 1]).to(dev)
    for s in range(0, len(rows), chunk):
        t0 = time.time()
        with torch.no_grad():
            _, _, n = model.forward_rows(h[s:s + chunk], r[s:s + chunk], None, return_ncand=True)
        torch.cuda.synchronize()
        print("rows %6d-%6d  %.3f s  scale %d  ncand max %d min %d" % (s, s + chunk, time.time() - t0,
              model.capacity_scale, int(n.max()), int(n.min())), flush=True)


if __name__ == "__main__":
    main()
