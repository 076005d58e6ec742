"""Diagnostic: forward_rows retry path, with variants (GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    graph, test_set, model, rows = bench.build_workload("bias")
    model = model.to(dev).eval()
    h = torch.from_numpy(rows[:, 0]).to(dev)
    r = torch.from_numpy(rows[:, 1]).to(dev)
    mode = sys.argv[1]
    if mode == "scale2":
        model.capacity_scale = 2
    if mode == "prealloc":
        model._workspace(dev, len(rows), 2)
    try:
        with torch.no_grad():
            s, m = model.forward_rows(h, r, None)
        torch.cuda.synchronize()
        print(mode, "OK scale", model.capacity_scale, flush=True)
    except Exception as e:
        print(mode, "FAIL", e, flush=True)


if __name__ == "__main__":
    main()
