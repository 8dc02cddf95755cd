#!/usr/bin/env python3
"""Where do renders of one k_final form differ from each other and from the
product form?  (Written for the prefetching form, SAMNERF_FINAL_PF=1 of the
round-3 diagnostic build, removed in round 4; with the switch gone every
render takes the product form.)  Renders the test_final_forms_deterministic view
several times with the parity taps and reports, per output and tap, how many
entries differ from the first render and the first few (ray, sample) places."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from helpers import make_net  # noqa: E402
from oracle import synth  # noqa: E402
from samnerf_amd import ops, _lib  # noqa: E402
from samnerf_amd.fused import FusedRenderer, ROW  # noqa: E402

dev = torch.device("cuda", 0)
os.environ["SAMNERF_FINAL_PF"] = os.environ.get("PF", "1")
os.environ["SAMNERF_FINAL_S"] = os.environ.get("SEG", "1")
spec = synth.ModelSpec(with_sam=True)
net = make_net(spec, synth.make_params(spec, seed=23, emb_scale=0.5, ln_jitter=0.1), dev)
pose, intr = synth.gui_camera(512, 80, rot=synth.random_rotation(11))
ro, rd = ops.get_rays(pose, intr, 80, 512, device=dev)
with _lib.diag_library():
    fr = FusedRenderer(net, head_mode=int(os.environ.get("HEAD_MODE", "0")))
    outs = []
    for _ in range(int(os.environ.get("REPS", "4"))):
        if os.environ.get("NEWFR") == "1":     # a fresh renderer (and workspace) per render
            fr = FusedRenderer(net, head_mode=int(os.environ.get("HEAD_MODE", "0")))
        rows = torch.empty(ro.shape[0], ROW, device=dev)
        o = fr.render(ro, rd, rows=rows, view_width=512, taps=True)
        o["rows"] = rows.clone()
        outs.append({k: v.clone() if torch.is_tensor(v) else v for k, v in o.items()})
        torch.cuda.synchronize()
# the product form (no prefetch) of the same view, for reference: which of
# the renders that differ is the odd one
os.environ["SAMNERF_FINAL_PF"] = "0"
with _lib.diag_library():
    rows = torch.empty(ro.shape[0], ROW, device=dev)
    o = FusedRenderer(net, head_mode=int(os.environ.get("HEAD_MODE", "0"))).render(
        ro, rd, rows=rows, view_width=512, taps=True)
    o["rows"] = rows.clone()
    ref = {k: v.clone() if torch.is_tensor(v) else v for k, v in o.items()}
for j, o in enumerate(outs):
    same = all(torch.equal(ref[k], o[k]) for k in ("image", "depth", "samvit", "sigma2"))
    print(f"render {j} equals the PF=0 render: {same}")
base = outs[0]
print({k: os.environ.get(k) for k in ("PF", "SEG", "HEAD_MODE", "NEWFR", "REPS")})
for j, o in enumerate(outs[1:], 1):
    print(f"render {j} vs 0:")
    for k, v in base.items():
        if not torch.is_tensor(v) or v.shape != o[k].shape:
            continue
        a, b = v, o[k]
        if a.dtype.is_floating_point:
            ne = ~((a == b) | (torch.isnan(a) & torch.isnan(b)))
        else:
            ne = a != b
        n = int(ne.sum())
        if n:
            idx = ne.nonzero()[:6].tolist()
            d = (a.double() - b.double()).abs()[ne].max().item() if a.dtype.is_floating_point else None
            print(f"  {k} {tuple(a.shape)}: {n} differ, max |d| {d}, first {idx}")
