#!/usr/bin/env python3
"""The --with_mask training step of bench.py (mask_train_steps: 4,096 rays,
'default' head, HIP kernels) alone, for a kernel trace:
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/mask_train_prof.py
prints ms per step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

ms, loss = bench.mask_train_steps(torch.device("cuda", 0), int(os.environ.get("STEPS", "20")), 5)
print({"ms_per_step": ms, "loss": loss})
