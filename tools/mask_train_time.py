#!/usr/bin/env python3
"""--with_mask training step time (bench.mask_train_steps: 4,096 rays, fused
HIP path vs the torch path).  usage (GPU box): python tools/mask_train_time.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

if __name__ == "__main__":
    import bench
    dev = torch.device("cuda", 0)
    ms, loss = bench.mask_train_steps(dev, 30, 5, fused=True)
    print(json.dumps({"fused_ms_per_step": ms, "loss": float(loss)}))
