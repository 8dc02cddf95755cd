#!/usr/bin/env python3
"""BASELINE config 5 (the SAM-distillation training step of bench.py
train_steps: 4,096 rays, HIP s_grid scatter, fused Adam) alone, for A/B runs
of library builds (SAMNERF_LIB): prints ms per step and the loss."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

ms, loss = bench.train_steps(torch.device("cuda", 0), int(os.environ.get("STEPS", "30")), 5)
print({"ms_per_step": ms, "loss": loss})
