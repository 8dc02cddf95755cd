#!/usr/bin/env python3
"""Five --with_mask training steps on the HIP path (bench.mask_train_steps),
for a kernel trace: rocprofv3 --kernel-trace --stats -- python3 tools/mask_train_prof.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import bench  # noqa: E402

ms, loss = bench.mask_train_steps(torch.device("cuda", 0), 5, 2, fused=len(sys.argv) < 2)
print({"ms_per_step": ms, "loss": loss})
