"""bf16x3 vs exact-fp32 renders of the bench view, row-major and tiled."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))
import bench  # noqa: E402
from samnerf_amd import ops, synth  # noqa: E402
from samnerf_amd.fused import FusedRenderer  # noqa: E402

dev = torch.device("cuda", 0)
net, _, _ = bench.build_net(True, dev)
pose, intr = synth.gui_camera(512, 512)
ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
outs = {}
for hm in (0, 1):
    for vw in (0, 512):
        o = FusedRenderer(net, head_mode=hm).render(ro, rd, view_width=vw)
        outs[(hm, vw)] = {k: v.cpu() for k, v in o.items()}
for k in ("image", "samvit"):
    print(k, "hm0 vs hm1 rowmajor", (outs[(0, 0)][k] - outs[(1, 0)][k]).abs().max().item(),
          "tiled", (outs[(0, 512)][k] - outs[(1, 512)][k]).abs().max().item(),
          "hm0 tiled vs rowmajor", (outs[(0, 0)][k] - outs[(0, 512)][k]).abs().max().item(),
          "hm1 tiled vs rowmajor", (outs[(1, 0)][k] - outs[(1, 512)][k]).abs().max().item())
