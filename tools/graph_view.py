#!/usr/bin/env python3
"""A render captured as a HIP graph (torch.cuda.CUDAGraph around
FusedRenderer.render: ray generation + the fused kernels, one graph launch
per view) against the eager launches, for the whole cfg3 view and one
rank's band at N = 8, interleaved rounds; checks the replayed outputs equal
the eager ones bit for bit.  usage (GPU box): python tools/graph_view.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))


def main():
    import bench
    from samnerf_amd import ops, synth
    from samnerf_amd.fused import FusedRenderer
    dev = torch.device("cuda", 0)
    net, _, _ = bench.build_net(True, dev)
    pose, intr = synth.gui_camera(512, 512)
    for rows in (64, 512):
        r0 = (512 - rows) // 2
        fr = FusedRenderer(net)

        def view():
            ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev, row0=r0, rows=rows)
            return fr.render(ro, rd, view_width=512)

        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(5):
                ref = view()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = view()
        g.replay()
        torch.cuda.synchronize()
        same = all(torch.equal(out[k], ref[k]) for k in ("image", "depth", "weights_sum", "samvit"))
        print(json.dumps({"rays": rows * 512, "graph_equals_eager": same}), flush=True)
        k = 60 if rows == 64 else 20
        for rnd in range(3):
            for mode in ("eager", "graph"):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(k):
                    if mode == "graph":
                        g.replay()
                    else:
                        view()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(json.dumps({"rays": rows * 512, "round": rnd, "mode": mode, "views": k,
                                  "enqueue_ms_per_view": (t1 - t0) * 1e3 / k,
                                  "ms_per_view": (t2 - t0) * 1e3 / k}), flush=True)
        del g


if __name__ == "__main__":
    main()
