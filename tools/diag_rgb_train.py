#!/usr/bin/env python3
"""Diagnostic (GPU box): where do the GPU RGB-training gradients and the CPU
twin's (tests/test_gpu_train.py) part?  Prints, per proposal stage, the
largest difference of the resampled bins, then loss and per-parameter
gradient errors, with the drop-in backward's row merging on and off."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "segment-anything-nerf_amd"), REPO, os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import nerf.renderer as R  # noqa: E402
from helpers import make_net  # noqa: E402
from oracle import renderer as orc  # noqa: E402
from oracle import synth  # noqa: E402
from oracle_backend import oracle_encoders  # noqa: E402
from samnerf_amd.train import rgb_train_step  # noqa: E402

rec = []
_orig = R.sample_pdf


def spy(bins, weights, T, perturb=False):
    out = _orig(bins, weights, T, perturb)
    rec.append((bins.detach().cpu(), weights.detach().cpu(), out.detach().cpu()))
    return out


R.sample_pdf = spy
cuda = torch.device("cuda:0")
spec = synth.ModelSpec(with_sam=False, grid_log2=12, s_grid_log2=10, prop_log2=10)
params = synth.make_params(spec, seed=12, emb_scale=0.5)
gpu = make_net(spec, params, cuda).train()
cpu = make_net(spec, params, "cpu").train()
pose, intr = synth.gui_camera(16, 16, rot=synth.random_rotation(6))
ro, rd = orc.get_rays(pose, intr, 16, 16)
gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(2))
_, lg, og = rgb_train_step(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda), global_step=1, perturb=False)
lg.backward()
rg = list(rec)
rec.clear()
with oracle_encoders():
    _, lc, oc = rgb_train_step(cpu, ro, rd, gt, global_step=1, perturb=False)
    lc.backward()
rc = list(rec)
for i, ((bg, wg, og_), (bc, wc, oc_)) in enumerate(zip(rg, rc)):
    print(f"stage {i}: |bins_in| {float((bg - bc).abs().max()):.3e}  |w| {float((wg - wc).abs().max()):.3e}"
          f"  |bins_out| {float((og_ - oc_).abs().max()):.3e}  rays with |bins_out|>1e-4: "
          f"{int(((og_ - oc_).abs().max(-1).values > 1e-4).sum())}")
print("loss gpu %.8f cpu %.8f" % (float(lg), float(lc)))
for k in ("proposal_loss", "distort_loss"):
    if k in og:
        print(k, float(og[k]), float(oc[k]))
print("max |weights| diff", float((og["weights"].detach().cpu() - oc["weights"].detach()).abs().max()))
print("max |image| diff", float((og["image"].detach().cpu() - oc["image"].detach()).abs().max()))
for (k, pg), (_, pc) in zip(gpu.named_parameters(), cpu.named_parameters()):
    if pc.grad is None:
        continue
    err = (pg.grad.cpu() - pc.grad).norm() / pc.grad.norm().clamp_min(1e-12)
    print(f"  {k:28s} rel {float(err):.3e}  max|d| {float((pg.grad.cpu() - pc.grad).abs().max()):.3e}"
          f"  max|g| {float(pc.grad.abs().max()):.3e}")
