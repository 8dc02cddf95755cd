"""N1 probe: the surface scene at 512x512 rendered in the default mode and
with t_thresh 1e-4, 10 times each (run under rocprofv3 --kernel-trace to
compare k_final<..., EXIT> with k_final)."""
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
net, _, _ = bench.build_net(True, dev, seed=3, surface=True)
pose, intr = synth.gui_camera(512, 512)
ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
dnet, _, _ = bench.build_net(True, dev)
# 10 renders per (scene, t): surface scene at t = 0, 1e-4, 0.5, 0.95; then the
# default-init scene at t = 0, 1e-4 (kernel trace order tells them apart)
for scene, n, ts in (("surface", net, (0.0, 1e-4, 0.5, 0.95)), ("default", dnet, (0.0, 1e-4))):
    for t in ts:
        r = FusedRenderer(n, t_thresh=t)
        for _ in range(10):
            out = r.render(ro, rd)
        torch.cuda.synchronize()
        ws = out["weights_sum"]
        print(scene, t, "rays with weights_sum < 1 - 1e-6:", (ws < 1 - 1e-6).float().mean().item(), flush=True)
