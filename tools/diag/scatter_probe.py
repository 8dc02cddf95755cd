"""How fast is the drop-in grid backward (k_grid_backward) on the torch RGB
step's own data, and how much of that is point order (samples along a ray
share corner rows, so the wave-level merge removes most atomics)?  Records
each grid_encode_backward call of one torch-path training step, then times
the drop-in kernel on it as recorded and with the points randomly permuted.
usage: python tools/diag/scatter_probe.py [N]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "segment-anything-nerf_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import gridencoder.grid as G  # noqa: E402
from helpers import make_net  # noqa: E402
from oracle import synth  # noqa: E402
from samnerf_amd import ops  # noqa: E402
from samnerf_amd.train import rgb_train_step  # noqa: E402


def main(N=8192):
    dev = torch.device("cuda:0")
    spec = synth.ModelSpec(with_sam=False)
    net = make_net(spec, synth.make_params(spec, seed=1, emb_scale=0.5), dev).train()
    net.fused = False                     # the torch path: run_torch + autograd + drop-in kernels
    side = int(round(N ** 0.5))
    pose, intr = synth.gui_camera(side, side, rot=synth.random_rotation(1))
    ro, rd = ops.get_rays(pose, intr, side, side, device=dev)
    gt = torch.rand(ro.shape[0], 3, device=dev)
    calls = []
    orig = G._backend.grid_encode_backward

    def rec(*args):
        calls.append([a.clone() if torch.is_tensor(a) else a for a in args])
        return orig(*args)
    G._backend.grid_encode_backward = rec
    _, loss, _ = rgb_train_step(net, ro, rd, gt, global_step=1)
    loss.backward()
    G._backend.grid_encode_backward = orig
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for ci, args in enumerate(calls):
        grad, inputs, emb, offs, gemb = args[:5]
        B, D, C, L = args[5:9]
        for mode in ("recorded", "permuted"):
            a = list(args)
            if mode == "permuted":
                perm = torch.randperm(B, device=dev)
                a[1] = inputs[perm].contiguous()
                a[0] = grad[:, perm].contiguous()
            times = []
            for it in range(6):
                a[4].zero_()
                ev[0].record()
                orig(*a)
                ev[1].record()
                torch.cuda.synchronize()
                times.append(ev[0].elapsed_time(ev[1]))
            print(json.dumps({"call": ci, "points": B, "levels": L, "mode": mode,
                              "ms": round(sorted(times)[len(times) // 2], 4)}))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
