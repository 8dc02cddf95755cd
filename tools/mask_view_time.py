#!/usr/bin/env python3
"""The --with_mask 'default' 512x512 view of bench.py (mask_view) alone, for
A/B runs of library builds (SAMNERF_LIB): prints ms per view and rays/s."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

r = bench.mask_view(torch.device("cuda", 0), 6, 2, 0, ref_rays=16384)
print(json.dumps({"ms_per_view": r["ms_per_step"], "rays_per_s": r["value"],
                  "max_abs_logits_vs_unfused": r["max_abs_logits_vs_unfused"],
                  "logits_sha16": r["logits_sha16"]}))
