"""Ray-order probe: the same 512x512 view rendered with its rays in row-major
order and permuted into tx x ty pixel tiles (each run of tx*ty consecutive
rays is one tile), on the default-init and the opaque-sphere scene; 10
renders per case (run under rocprofv3 --kernel-trace)."""
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
H = W = 512
pose, intr = synth.gui_camera(W, H)
ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
TILES = [(32, 1), (16, 2), (8, 4), (8, 8), (16, 4)]


def perm(tx, ty):
    idx = torch.arange(H * W, device=dev).view(H // ty, ty, W // tx, tx)
    return idx.permute(0, 2, 1, 3).reshape(-1)


for scene in ("default", "surface"):
    net, _, _ = bench.build_net(True, dev, seed=3 if scene == "surface" else 0, surface=scene == "surface")
    r = FusedRenderer(net)
    ref = None
    for tx, ty in TILES:
        p = perm(tx, ty)
        for _ in range(10):
            out = r.render(ro[p].contiguous(), rd[p].contiguous())
        torch.cuda.synchronize()
        img = torch.empty_like(out["image"])
        img[p] = out["image"]
        if ref is None:
            ref = img
        print(scene, tx, ty, "max |image - row-major|", (img - ref).abs().max().item(), flush=True)
