"""WN18RR (config 3) forward steps for rocprofv3 (diagnostic; GPU box):
rocprofv3 --kernel-trace --stats -- python tools/wn_profile.py [feature]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(bench.wn18rr_line(torch.device("cuda:0"), reps=5))
