#!/usr/bin/env python3
"""Which path k_sgrid_box4 takes (its phase budget): per
(wave, sample, level) the uniform-cell path (8 corner rows through the
scalar cache), the staged box (distinct rows into LDS, 8 corners per lane
from LDS) or direct gathers (box over kBoxSlots), and the staged boxes' mean
slots / cells -- counted by the diagnostic build (SAMNERF_SGRID_PATHS) on a
whole 512^2 cfg3 view of the bench's default scene and of the opaque-sphere
scene.  usage (GPU box): python tools/sgrid_paths.py"""
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
    dev = torch.device("cuda", 0)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
    for scene in ("default", "surface"):
        net, _, _ = bench.build_net(True, dev, surface=scene == "surface")
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        os.environ["SAMNERF_SGRID_PATHS"] = f"{cnt.data_ptr():x}"
        try:
            with _lib.diag_library():
                FusedRenderer(net).render(ro, rd, view_width=512)
                torch.cuda.synchronize()
        finally:
            os.environ.pop("SAMNERF_SGRID_PATHS", None)
        c = cnt.cpu().tolist()
        ev = c[0] + c[1] + c[2]
        print(json.dumps({"scene": scene, "wave_sample_levels": ev,
                          "uniform": c[0] / max(ev, 1), "box": c[1] / max(ev, 1), "direct": c[2] / max(ev, 1),
                          "skipped_wave_samples": c[3],
                          "box_mean_slots": c[4] / max(c[1], 1), "box_mean_cells": c[5] / max(c[1], 1)}),
              flush=True)


if __name__ == "__main__":
    main()
