#!/usr/bin/env python3
"""A/B of SAM-head forms inside the headline view (512x512, RGB + SAM
feature): view time with the product library vs the diagnostic build at
SAMNERF_HEAD_V=<form>, interleaved rounds so clock / thermal drift hits both.
usage (GPU box): python tools/head_view_ab.py FORM [rounds] [views]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))


def main():
    import bench
    from samnerf_amd import _lib, ops, synth
    from samnerf_amd.fused import FusedRenderer
    form = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    views = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    net, _, _ = bench.build_net(True, dev)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)

    def timed(diag):
        os.environ["SAMNERF_HEAD_V"] = form
        ctx = _lib.diag_library() if diag else _nullctx()
        with ctx:
            fr = FusedRenderer(net)
            out = fr.render(ro, rd, view_width=512)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(views):
                fr.render(ro, rd, view_width=512)
            e1.record()
            torch.cuda.synchronize()
        os.environ.pop("SAMNERF_HEAD_V")
        return out, e0.elapsed_time(e1) / views

    res = {"form": form, "product_ms": [], "form_ms": []}
    base = None
    for _ in range(rounds):
        o, ms = timed(False)
        res["product_ms"].append(round(ms, 4))
        base = o if base is None else base
        o2, ms2 = timed(True)
        res["form_ms"].append(round(ms2, 4))
        res["bit_identical"] = all(torch.equal(o2[k], base[k]) for k in base)
    res["product_mean"] = sum(res["product_ms"]) / rounds
    res["form_mean"] = sum(res["form_ms"]) / rounds
    print(json.dumps(res))


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
