#!/usr/bin/env python3
"""A/B of one diagnostic switch inside the headline view: view time with the
product library vs the diagnostic build with NAME=VALUE set, interleaved
rounds so clock / thermal drift hits both, on the default or the
opaque-sphere scene.  usage (GPU box):
  python tools/view_ab.py NAME=VALUE [--surface] [--rounds 5] [--views 20]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))


def main():
    import contextlib
    import bench
    from samnerf_amd import _lib, ops, synth
    from samnerf_amd.fused import FusedRenderer
    ap = argparse.ArgumentParser()
    ap.add_argument("switch")
    ap.add_argument("--surface", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--views", type=int, default=20)
    a = ap.parse_args()
    name, value = a.switch.split("=", 1)
    dev = torch.device("cuda", 0)
    net, _, _ = bench.build_net(True, dev, surface=a.surface)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)

    def timed(diag):
        os.environ[name] = value
        with (_lib.diag_library() if diag else contextlib.nullcontext()):
            fr = FusedRenderer(net)
            out = fr.render(ro, rd, view_width=512)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.views):
                fr.render(ro, rd, view_width=512)
            e1.record()
            torch.cuda.synchronize()
        os.environ.pop(name)
        return out, e0.elapsed_time(e1) / a.views

    res = {"switch": a.switch, "scene": "surface" if a.surface else "default", "product_ms": [], "diag_ms": []}
    base = None
    for _ in range(a.rounds):
        o, ms = timed(False)
        res["product_ms"].append(round(ms, 4))
        base = o if base is None else base
        o2, ms2 = timed(True)
        res["diag_ms"].append(round(ms2, 4))
        res["bit_identical"] = all(torch.equal(o2[k], base[k]) for k in base)
    res["product_mean"] = sum(res["product_ms"]) / a.rounds
    res["diag_mean"] = sum(res["diag_ms"]) / a.rounds
    print(json.dumps(res))


if __name__ == "__main__":
    main()
