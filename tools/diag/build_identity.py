"""Diagnostic: render views with the library named by SAMNERF_LIB (or the
in-tree build) and save every output; `compare a.npz b.npz` checks that two
builds give identical bits (a kernel change meant to keep them)."""
import os
import sys

import numpy as np

if sys.argv[1] == "compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
    for k in bad:
        print("DIFF", k, float(np.nanmax(np.abs(a[k] - b[k]))))
    print("identical" if not bad else f"{len(bad)} outputs differ", len(a.files), "outputs")
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "segment-anything-nerf_amd"), os.path.join(REPO, "tests")]
from helpers import make_net  # noqa: E402
from samnerf_amd import ops, synth  # noqa: E402
from samnerf_amd.fused import FusedRenderer, ROW  # noqa: E402

cuda = torch.device("cuda:0")
res = {}
for tag, seed, es, n in (("parity", 23, 0.5, 262144), ("default", 0, 1e-4, 262144), ("share", 23, 0.5, 32768)):
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=seed, emb_scale=es, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(512, 512, rot=synth.random_rotation(seed + 5))
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=cuda)
    rd[1000] = float("nan")                      # a NaN ray (NaN positions in every kernel)
    rd[2000, 1] = float("inf")
    rows = torch.empty(n, ROW, device=cuda)
    o = FusedRenderer(net).render(ro[:n], rd[:n], rows=rows)
    torch.cuda.synchronize()
    for k, v in o.items():
        res[f"{tag}_{k}"] = v.float().cpu().numpy()
    res[f"{tag}_rows"] = rows.cpu().numpy()
np.savez(sys.argv[1], **res)
print("saved", sys.argv[1], len(res))
