"""Config 3's training step on the GPU box (bench.wn18rr_train_line): the
PNA statistics on the HIP path against the autograd-COO path."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.wn18rr_train_line(torch.device("cuda:0"))))
