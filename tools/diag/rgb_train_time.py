"""Time one RGB training step (nerf/utils.py:897-937, BASELINE-style synthetic
scene at the reference's table sizes) on the HIP training kernels
(rgb_train_step_fused) against the torch path (rgb_train_step + autograd),
both with FusedAdam.  usage: python tools/diag/rgb_train_time.py [N ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "segment-anything-nerf_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from helpers import make_net  # noqa: E402
from oracle import synth  # noqa: E402
from samnerf_amd import ops  # noqa: E402
from samnerf_amd.optim import FusedAdam  # noqa: E402
from samnerf_amd.train import rgb_train_step, rgb_train_step_fused  # noqa: E402


def run(N, fused, steps=20, warmup=5):
    dev = torch.device("cuda:0")
    spec = synth.ModelSpec(with_sam=False)
    net = make_net(spec, synth.make_params(spec, seed=1, emb_scale=0.5), dev).train()
    net.opt.adaptive_num_rays = False
    net.fused = fused          # False: NeRFRenderer.run_torch under autograd
    opt = FusedAdam(net.get_params(1e-2), eps=1e-15)
    side = int(round(N ** 0.5))
    pose, intr = synth.gui_camera(side, side, rot=synth.random_rotation(1))
    ro, rd = ops.get_rays(pose, intr, side, side, device=dev)
    gt = torch.rand(ro.shape[0], 3, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(warmup + steps):
        if i == warmup:
            torch.cuda.synchronize()
            ev[0].record()
        if fused:
            _, loss, _ = rgb_train_step_fused(net, ro, rd, gt, global_step=1 + i)
        else:
            _, loss, _ = rgb_train_step(net, ro, rd, gt, global_step=1 + i)
            for p in net.parameters():
                p.grad = None
            loss.backward()
        opt.step()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / steps
    return {"rays": ro.shape[0], "fused": fused, "ms_per_step": ms, "rays_per_s": ro.shape[0] / ms * 1e3,
            "final_loss": float(loss)}


if __name__ == "__main__":
    sizes = [int(v) for v in sys.argv[1:]] or [4096, 8192]
    for N in sizes:
        a, b = run(N, True), run(N, False)
        a["speedup_vs_torch_path"] = b["ms_per_step"] / a["ms_per_step"]
        print(json.dumps(a))
        print(json.dumps(b))
