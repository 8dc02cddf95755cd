#!/usr/bin/env python3
"""Ray-tile order (SAMNERF_SUPERTILE, read by the diagnostic build only) on the
default-init and the opaque-sphere 512x512 views: view time per supertile
width and bit-identity of the outputs against the plain 8x4 tiling.
usage (GPU box): python tools/tile_order_bench.py [widths, default 0,4,8,16]"""
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
    widths = (sys.argv[1] if len(sys.argv) > 1 else "0,4,8,16").split(",")
    dev = torch.device("cuda", 0)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
    res = {}
    for scene in ("default", "surface"):
        net, _, _ = bench.build_net(True, dev, surface=scene == "surface")
        fr = FusedRenderer(net)
        base = None
        for sw in widths:
            os.environ["SAMNERF_SUPERTILE"] = sw
            with _lib.diag_library():
                out = fr.render(ro, rd, view_width=512)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fr.render(ro, rd, view_width=512)
                e1.record()
                torch.cuda.synchronize()
            if base is None:
                base = out
            same = all(torch.equal(out[k], base[k]) for k in base)
            res[f"{scene}_sw{sw}"] = {"ms": e0.elapsed_time(e1) / 10, "bit_identical": same}
    os.environ.pop("SAMNERF_SUPERTILE", None)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
