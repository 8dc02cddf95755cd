#!/usr/bin/env python3
"""N1 (flagged early-exit mode) on the opaque-sphere scene at 512x512: view
time and final-stage time of the default mode and of N1 at several
t_thresh, for each chunk count of the ray compaction (SAMNERF_N1_CHUNKS, read
by the diagnostic build only; 1 = the wave-level exit alone), with the error
against the default mode.  usage (GPU box): python tools/n1_bench.py
"""
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
    net, _, _ = bench.build_net(True, dev, surface=True)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)

    def timed(fr, iters=10):
        out = fr.render(ro, rd, view_width=512)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fr.render(ro, rd, view_width=512)
        e1.record()
        torch.cuda.synchronize()
        return out, e0.elapsed_time(e1) / iters

    res = {}
    full, ms = timed(FusedRenderer(net))
    res["default_ms"] = ms
    for t in (1e-4, 1e-3, 1e-2):
        for c in ("1", "2", "4", "8"):
            os.environ["SAMNERF_N1_CHUNKS"] = c
            with _lib.diag_library():
                out, ms = timed(FusedRenderer(net, t_thresh=t))
            res[f"t{t:g}_c{c}"] = {
                "ms": ms,
                "wsum_drop": (full["weights_sum"] - out["weights_sum"]).max().item(),
                "closed_rays": (out["weights_sum"] != full["weights_sum"]).float().mean().item(),
                "samvit_err": (full["samvit"] - out["samvit"]).abs().max().item()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
