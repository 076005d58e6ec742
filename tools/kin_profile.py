"""kinship (config 2) forward steps for rocprofv3 / A/B runs (diagnostic; GPU box):
python tools/kin_profile.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(bench.kinship_line(torch.device("cuda:0"), reps=20))
