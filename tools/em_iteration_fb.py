"""One EM iteration of run_rnnlogic.py (config/FB15k-237.yaml) on FB15k-237,
timed per phase on one GPU — bench.py's `em_iteration` line on its own.
Usage (GPU box): python tools/em_iteration_fb.py [PRE_EPOCHS]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    pre = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    print(json.dumps(bench.em_iteration_line(torch.device("cuda:0"), pre)), flush=True)
