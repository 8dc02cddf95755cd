#!/usr/bin/env python3
"""Host cost of issuing one render against the GPU time of one render: for
the whole cfg3 view (262,144 rays) and one rank's band at N = 8 (32,768
rays), the wall time of enqueueing K renders (no synchronisation; the queue
absorbs them) against the wall time until they finish.  A band render whose
enqueue time approaches its GPU time is host-bound, and that is what a
captured HIP graph (one launch per view) removes.  usage (GPU box):
python tools/host_overhead.py"""
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
    for rows in (512, 64):
        r0 = (512 - rows) // 2
        ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev, row0=r0, rows=rows)
        fr = FusedRenderer(net)
        for _ in range(5):
            fr.render(ro, rd, view_width=512)
        torch.cuda.synchronize()
        for k in (10, 30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                fr.render(ro, rd, view_width=512)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"rays": rows * 512, "views": k, "enqueue_ms_per_view": (t1 - t0) * 1e3 / k,
                              "ms_per_view": (t2 - t0) * 1e3 / k}), flush=True)
        # host cost of the Python side alone: the same calls with the GPU idle
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fr.render(ro, rd, view_width=512)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(json.dumps({"rays": rows * 512, "one_call_enqueue_ms_idle_gpu": (t1 - t0) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
