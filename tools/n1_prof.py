#!/usr/bin/env python3
"""Five N1 renders (t_thresh 1e-4) of the opaque-sphere 512x512 view through
the diagnostic build (SAMNERF_N1_CHUNKS from the environment), for a kernel
trace (tools/n1_prof.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import bench  # noqa: E402
from samnerf_amd import _lib, ops, synth  # noqa: E402
from samnerf_amd.fused import FusedRenderer  # noqa: E402

dev = torch.device("cuda", 0)
net, _, _ = bench.build_net(True, dev, surface=True)
pose, intr = synth.gui_camera(512, 512)
ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
with _lib.diag_library():
    fr = FusedRenderer(net, t_thresh=1e-4)
    for _ in range(5):
        fr.render(ro, rd, view_width=512)
torch.cuda.synchronize()
