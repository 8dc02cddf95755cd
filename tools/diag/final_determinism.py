"""Diagnostic: k_final outputs for PF on/off, repeated, at one N (S form by N)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "segment-anything-nerf_amd"), os.path.join(REPO, "tests")]
from helpers import make_net  # noqa: E402
from oracle import synth  # noqa: E402
from samnerf_amd import ops  # noqa: E402
from samnerf_amd.fused import FusedRenderer, ROW  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 70000
cuda = torch.device("cuda:0")
spec = synth.ModelSpec(with_sam=True)
net = make_net(spec, synth.make_params(spec, seed=23, emb_scale=0.5, ln_jitter=0.1), cuda)
pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(11))
ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)
fr = FusedRenderer(net)
outs = {}
for pf in ("0", "1", "0", "1"):
    os.environ["SAMNERF_FINAL_PF"] = pf
    rows = torch.empty(n, ROW, device=cuda)
    o = fr.render(ro[:n], rd[:n], rows=rows)
    torch.cuda.synchronize()
    outs.setdefault(pf, []).append({k: v.clone() for k, v in o.items()} | {"rows": rows.clone()})
for pf in ("0", "1"):
    a, b = outs[pf]
    print("PF", pf, "repeat equal:", {k: bool(torch.equal(a[k], b[k])) for k in a})
a, b = outs["0"][0], outs["1"][0]
for k in a:
    d = (a[k] - b[k]).abs()
    if d.dim() > 1:
        d = d.amax(dim=1)
    bad = torch.nonzero(d > 0).flatten()
    print("PF0 vs PF1", k, "max", d.max().item(), "rays differing", bad.numel(), bad[:10].tolist())
