#!/usr/bin/env python3
"""Fingerprints of the outputs of one library build (SAMNERF_LIB, or the
in-tree product): the headline view on the default and the parity-weight
scene, the sphere scene, the --with_mask view and one mask-training forward,
as sha256 prefixes of the raw bytes.  Two builds whose lines match are
bit-identical on these workloads (A/B of kernel forms that must keep the
bits).  usage (GPU box): [SAMNERF_LIB=...] python tools/lib_bits.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def sha(t):
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    from samnerf_amd import ops, synth
    from samnerf_amd.fused import FusedRenderer
    dev = torch.device("cuda", 0)
    H = W = 512
    pose, intr = synth.gui_camera(W, H)
    ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
    out = {}
    for tag, kw in (("default", {}), ("parity", {"emb_scale": 0.5}), ("sphere", {"surface": True, "seed": 3})):
        for head_mode in (0, 1):
            if tag != "default" and head_mode == 1:
                continue
            net, _, _ = bench.build_net(True, dev, **kw)
            o = FusedRenderer(net, head_mode=head_mode).render(ro, rd, view_width=W)
            out[f"{tag}_h{head_mode}"] = {k: sha(o[k]) for k in ("image", "depth", "samvit")}
    r = bench.mask_view(dev, 1, 1, 0, ref_rays=16384)
    out["mask_logits"] = r["logits_sha16"]
    _, loss = bench.mask_train_steps(dev, 1, 0)          # the first step's forward loss (before any update)
    out["mask_train_loss"] = float(loss).hex()
    print(json.dumps(out, sort_keys=True))


if __name__ == "__main__":
    main()
